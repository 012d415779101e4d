"""oracle/encfm.py's cnn / swin meta-encoders (fixed steps) against tests/golden/kd_encfm_meta.npz,
made from the reference's own FlowMatchingModule / SwinTransformerEncoder (make_golden_encfm_meta.py,
asr_train.py:844-866, 1220-1377): losses rtol 1e-5, FM output and every gradient (all parameters, every
hooked student layer) max|diff| <= 1e-5 * max|ref| + 1e-7.  Also the engine's parameter specs
(kdfm/config.py meta_specs) against the fixture's names / shapes, and the configurations the engine
refuses."""
from dataclasses import replace

import numpy as np
import pytest
import torch

import encfm_meta_fixture as FX
from oracle import encfm as E


@pytest.mark.parametrize("meta", ["cnn", "swin", "conformer", "unet"])
def test_meta_oracle_matches_reference(meta):
    z = FX.load()
    steps = [int(x) for x in z["meta.steps"]]
    P = {k: v.double().requires_grad_(True) for k, v in FX.params(z, meta).items()}
    s, t, R = FX.inputs(z, T=z.get(meta + ".meta.T"))
    s = [x.double().requires_grad_(True) for x in s]
    bn = FX.bn_init(z, meta)
    out = E.encfm_fixed_forward(P, s, [x.double() for x in t], steps, meta=meta, heads=2, bn_state=bn)
    for k, v in bn.items():   # BatchNorm running statistics after sum(steps) module calls
        np.testing.assert_allclose(v.numpy(), z[meta + ".buffer." + k], rtol=1e-5, atol=1e-7)
    pre = meta + "."
    np.testing.assert_allclose(float(out["total"].detach()), float(z[pre + "total"]), rtol=1e-5)
    np.testing.assert_allclose([float(x.detach()) for x in out["flow"]], z[pre + "flow"], rtol=1e-5)

    def close(a, b, what):
        a = a.detach().double().numpy()
        err = np.abs(a - b).max()
        assert err <= 1e-5 * np.abs(b).max() + 1e-7, f"{what}: {err:.3e} vs max {np.abs(b).max():.3e}"

    close(out["fm_out"], z[pre + "fm_out"], "fm_out")
    obj = out["total"] + (out["fm_out"] * R.double()).sum()
    names = list(P)
    grads = torch.autograd.grad(obj, [P[n] for n in names] + s, allow_unused=True)
    for n, g in zip(names, grads):
        g = torch.zeros_like(P[n]) if g is None else g
        if n.endswith("depthwise_conv.bias"):
            # analytically zero: BatchNorm with batch statistics removes a per-channel shift; the fixture
            # holds float32 rounding residue (~1e-5), the float64 oracle ~1e-16
            assert np.abs(z[pre + "grad." + n]).max() < 1e-4 and g.abs().max().item() < 1e-4, n
            continue
        close(g, z[pre + "grad." + n], n)
    for i in range(len(s)):
        close(grads[len(names) + i], z[pre + f"grad.s{i}"], f"s{i}")


@pytest.mark.parametrize("meta", ["cnn", "swin", "conformer", "unet"])
def test_meta_specs_match_reference(meta):
    from kdfm.config import DEFAULT, encfm_specs
    z = FX.load()
    cfg = replace(DEFAULT, kd_model="encfm", encfm_meta=meta, encfm_dynamic=False,
                  encfm_steps_per_layer=(2,) * DEFAULT.n_layers, encfm_hidden=int(z.get(meta + ".meta.hidden", 128)))
    specs = encfm_specs(cfg)
    assert [n for n, _ in specs] == [str(n) for n in z[meta + ".names"]]
    assert [str(tuple(s)) for _, s in specs] == [str(s) for s in z[meta + ".shapes"]]


def test_meta_refusals():
    from kdfm.config import DEFAULT, head_specs
    with pytest.raises(ValueError, match="fixed step counts"):
        head_specs(replace(DEFAULT, kd_model="encfm", encfm_meta="cnn", encfm_dynamic=True))
    for meta in ("bogus",):
        with pytest.raises(ValueError, match="encfm_meta"):
            head_specs(replace(DEFAULT, kd_model="encfm", encfm_meta=meta, encfm_dynamic=False,
                               encfm_steps_per_layer=(2,) * DEFAULT.n_layers))


def test_unet_odd_frames_fail_like_the_reference():
    """UNet1D returns 2 floor(T / 2) frames: at an odd T the reference's update x - v / S cannot broadcast
    (asr_train.py:1340-1358); the oracle raises there too (the engine refuses the shape, test_encfm_meta_gpu)."""
    z = FX.load()
    P = {k: v.double() for k, v in FX.params(z, "unet").items()}
    s, t, _ = FX.inputs(z, T=35)
    with pytest.raises(RuntimeError, match="size of tensor"):
        E.fm_forward(P, s[0].double(), t[0].double(), 2, meta="unet")
