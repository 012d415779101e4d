"""Pin the oracle's KD heads to vectors produced by the reference's own classes
(tests/golden/make_golden.py; asr_train_diffm.py:400-497, 645-702, 852-856, 1270-1427)."""
import os

import numpy as np
import pytest
import torch

from oracle import ver5

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_heads_ver5.npz")
# one benchmark-shape layer (B=1, T'=401 = 16.0 s after 4x subsampling), same generator
GOLD_BENCH = os.path.join(os.path.dirname(__file__), "golden", "kd_heads_ver5_b1t401.npz")


@pytest.fixture(scope="module", params=[GOLD, GOLD_BENCH], ids=["b2t29", "b1t401"])
def gold(request):
    return dict(np.load(request.param, allow_pickle=False))


def _params(gold):
    return {k[len("param."):]: torch.tensor(v, requires_grad=True) for k, v in gold.items() if k.startswith("param.")}


def test_heads_forward_matches_reference(gold):
    cfg = ver5.StepConfig()
    p = _params(gold)
    s = torch.tensor(gold["in.s"], requires_grad=True)
    t = torch.tensor(gold["in.t"])
    eps = torch.tensor(gold["in.eps"])
    recon, fm = ver5.ver5_layer_losses(s, t, p, eps, cfg)
    assert abs(recon.item() - float(gold["out.recon"])) <= 1e-6 * max(1.0, abs(float(gold["out.recon"])))
    assert abs(fm.item() - float(gold["out.fm_post"])) <= 1e-6 * max(1.0, abs(float(gold["out.fm_post"])))
    names = [k for k in p if not k.startswith("fm_latent_2.")]
    grads = torch.autograd.grad(recon + fm, [p[n] for n in names] + [s])
    for n, g in zip(names, grads[:-1]):
        np.testing.assert_allclose(g.numpy(), gold["grad." + n], rtol=1e-5, atol=1e-6, err_msg=n)
    np.testing.assert_allclose(grads[-1].numpy(), gold["grad.in.s"], rtol=1e-5, atol=1e-6)


def test_denoiser_and_fm_x_match_reference(gold):
    if "out.z_deno" not in gold:
        pytest.skip("the benchmark-shape fixture records losses and gradients only")
    cfg = ver5.StepConfig()
    p = {k: v.detach() for k, v in _params(gold).items()}
    s = torch.tensor(gold["in.s"]).transpose(1, 2)
    t = torch.tensor(gold["in.t"]).transpose(1, 2)
    eps = torch.tensor(gold["in.eps"])
    z = ver5.sproj(s, p)
    zn, g = ver5.noise_adapter(z, p, eps)
    np.testing.assert_allclose(g.numpy(), gold["out.gamma"], rtol=1e-6, atol=1e-7)
    zd = ver5.denoiser(zn, p, cfg.denoiser_steps)
    np.testing.assert_allclose(zd.numpy(), gold["out.z_deno"], rtol=1e-5, atol=1e-6)
    zt, _ = ver5.tae(t, p)
    _, x = ver5.fm_latent(zd, zt, p, cfg.fm_steps)
    np.testing.assert_allclose(x.numpy(), gold["out.fm_x"], rtol=1e-5, atol=1e-6)
