"""The cnn / swin FM meta-encoders on the engine (kdfm/fmmeta.py) against (a) tests/golden/
kd_encfm_meta.npz, made from the reference's own FlowMatchingModule / SwinTransformerEncoder
(make_golden_encfm_meta.py; asr_train.py:844-866, 1220-1377), and (b) the whole training step of the
asr_train.py family with that meta-encoder vs oracle/ver5.py (fixed steps) in float64.

The meta-encoder GEMMs run bf16 MFMA with f32 state (the swin attention is the fused bf16 attention
pair): flow losses rtol 2e-2, FM output and every FM / feature gradient relative Frobenius <= 3e-2 (the
tolerance of the other bf16 FM chains); whole step as test_encfm_gpu.py (losses rtol 2e-2, gradients
relative Frobenius <= 5e-2)."""
from dataclasses import replace

import numpy as np
import pytest
import torch

import encfm_meta_fixture as FX

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("meta", ["cnn", "swin"])
def test_meta_matches_reference(meta):
    from kdfm import kernels as K
    from kdfm.config import DEFAULT, encfm_specs
    from kdfm.encfm import encfm_backward, encfm_forward
    from kdfm.fmmeta import MetaFMWorkspace
    z = FX.load()
    L, B, T = int(z["meta.L"]), int(z["meta.B"]), int(z["meta.T"])
    steps = tuple(int(x) for x in z["meta.steps"])
    cfg = replace(DEFAULT, n_layers=L, kd_model="encfm", encfm_meta=meta, encfm_dynamic=False,
                  encfm_steps_per_layer=steps, heads_student=2)
    dev = torch.device("cuda")
    P = {k: v.to(dev).contiguous() for k, v in FX.params(z, meta).items()}
    s, t, R = FX.inputs(z)
    sd = torch.stack([x.reshape(B * T, -1) for x in s]).to(dev).contiguous()
    td = torch.stack([x.reshape(B * T, -1) for x in t]).to(dev).contiguous()
    Rd = R.reshape(B * T, -1).to(dev).contiguous()
    G = {n: torch.zeros(shape, device=dev) for n, shape in encfm_specs(cfg)}
    ws = MetaFMWorkspace(cfg, B, T, dev)
    with K.mode("bf16", True):
        encfm_forward(cfg, P, sd, td, ws, train=True)
        dfeats = torch.empty(L * B * T, cfg.d_student, device=dev)
        encfm_backward(cfg, P, G, ws, dfeats, Rd, lambda fn, *keep: fn())
    torch.cuda.synchronize()
    pre = meta + "."
    np.testing.assert_allclose(ws.flow.cpu().numpy(), z[pre + "flow"], rtol=2e-2)
    np.testing.assert_allclose(ws.stats[2].item(), float(z[pre + "total"]), rtol=2e-2)
    assert _rel(ws.xS.view(B, T, -1), z[pre + "fm_out"]) <= 3e-2
    d = dfeats.view(L, B, T, -1)
    for i in range(L):
        r = _rel(d[i], z[pre + f"grad.s{i}"])
        assert r <= 3e-2, f"d/ds layer {i}: {r:.3e}"
    bad = []
    for n, gr in G.items():
        r = _rel(gr, z[pre + "grad." + n])
        if r > 3e-2:
            bad.append(f"{n}: {r:.3e}")
    assert not bad, bad


@pytest.mark.parametrize("meta", ["cnn", "swin"])
def test_meta_engine_step_matches_oracle(meta):
    import test_step_parity_gpu as SP
    from oracle import ver5 as O
    n_layers, B, N = 2, 2, 19200
    steps = (2, 3)
    cfg, eng, wav, wl, tg, tgl, g = SP._build(n_layers, B, N, [19200, 16123], 12, [12, 7],
                                              sub=dict(kd_model="encfm", encfm_dynamic=False, encfm_meta=meta,
                                                       encfm_steps_per_layer=steps))
    ctx = eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True)
    losses = eng.losses.detach().cpu().clone()
    eng.backward(ctx)
    torch.cuda.synchronize()
    grads = eng.student.grads()
    ocfg, p32 = SP._oracle_params(cfg, eng)
    ocfg.kd_model, ocfg.encfm_fixed, ocfg.encfm_meta = "encfm", steps, meta
    p = {k: (v.double() if v.is_floating_point() else v) for k, v in p32.items()}
    names = O.trainable_names(p, cfg.version, cfg.use_diffkd)
    names = [k for k in names if not k.startswith(("tae.", "sproj.", "adapter.", "denoiser.", "fm_latent", "router."))]
    for k in names:
        p[k] = p[k].clone().requires_grad_(True)
    out = O.ver5_step(p, wav.double(), wl, tg, tgl, ocfg, None)
    ref = torch.stack([out["loss"], out["ctc"], out["kl"], out["recon"], out["fm"]]).detach().float()
    torch.testing.assert_close(losses, ref, rtol=2e-2, atol=1e-3)
    og = torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
    bad = []
    for k, gr in zip(names, og):
        gr = torch.zeros_like(p[k]) if gr is None else gr
        if k.endswith(SP.ANALYTIC_ZERO) or gr.norm() == 0:
            continue
        r = _rel(grads[k], gr)
        if r > 5e-2:
            bad.append(f"{k}: {r:.3e}")
    assert not bad, bad
