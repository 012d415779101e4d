"""KD versions 1-8 through the module API on the GPU (kdfm.distill: kernel-backed TeacherAutoEncoder,
StudentProjector, NoiseAdapter, SimpleDenoiser, FMLatent x2, MSE/L1 kd_crit) against golden vectors
from the reference's own `_compute_v_losses_one_layer` (tests/golden/make_golden_versions.py,
asr_train_diffm.py:645-729).  fp32 MFMA parity mode; tolerances as the ver5 head tests."""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_heads_versions.npz")
KEYS = ("recon_loss", "kd_loss_pre", "fm_loss_pre", "kd_loss_post", "fm_loss_post")
CASES = [(v, "mse") for v in range(1, 9)] + [(1, "l1"), (3, "l1"), (8, "l1")]


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _heads(gold, version, kd):
    from kdfm import distill as Dm

    class Heads(nn.Module):   # the attributes DistilFlowMatchingCTCModelBPE builds for the heads
        _USES = Dm.DistilFlowMatchingCTCModelBPE._USES

        def __init__(self):
            super().__init__()
            flow = {"hidden_dim": 96, "shape_transform": "linear"}
            self.version = version
            self.kd_crit = Dm.l1_loss if kd == "l1" else Dm.mse_loss
            self.tae = Dm.TeacherAutoEncoder(176, 96)
            self.sproj = Dm.StudentProjector(88, 96)
            self.adapter = Dm.NoiseAdapter(96)
            self.denoiser = Dm.SimpleDenoiser(96, steps=9)
            self.fm_latent = Dm.FMLatent(96, flow)
            self.fm_latent_2 = Dm.FMLatent(96, flow)

    h = Heads()
    sd = {k[len("param."):]: torch.tensor(v) for k, v in gold.items() if k.startswith("param.")}
    h.load_state_dict(sd, strict=True)
    return h.cuda().train()


@pytest.mark.parametrize("version,kd", CASES)
def test_module_versions_match_reference(gold, version, kd):
    from kdfm import kernels as K
    from kdfm.distill import DistilFlowMatchingCTCModelBPE as M

    K.set_math("f32")
    h = _heads(gold, version, kd)
    B, T = int(gold["meta.B"]), int(gold["meta.T"])
    eps = torch.tensor(gold["in.eps"]).transpose(1, 2).reshape(B * T, 96).contiguous().cuda()
    h.adapter.eps_override = eps
    s = torch.tensor(gold["in.s"]).cuda().requires_grad_(True)
    t = torch.tensor(gold["in.t"]).cuda()
    out = M._compute_v_losses_one_layer(h, s, t)
    tag = f"v{version}{kd}"
    for k in KEYS:
        np.testing.assert_allclose(float(out[k]), float(gold[f"{tag}.{k}"]), rtol=2e-4, atol=1e-6, err_msg=k)
    total = sum(out[k] for k in KEYS)
    params = dict(h.named_parameters())
    names = list(params)
    grads = torch.autograd.grad(total, [params[n] for n in names] + [s], allow_unused=True)
    gs = grads[-1].cpu().numpy()
    ref = gold[f"{tag}.grad.s"]
    assert np.abs(gs - ref).max() <= 2e-3 * np.abs(ref).max() + 1e-6
    for n, g in zip(names, grads[:-1]):
        g = torch.zeros_like(params[n]) if g is None else g
        got = np.array([float(g.double().sum()), float((g.double() ** 2).sum())])
        r = gold[f"{tag}.gsum.{n}"]
        if r[1] == 0.0:
            assert got[1] == 0.0, n       # parameter off this version's path: exactly no gradient
            continue
        np.testing.assert_allclose(got[1], r[1], rtol=5e-3, err_msg=n)
        assert abs(got[0] - r[0]) <= 5e-3 * abs(r[0]) + 2e-3 * np.sqrt(r[1] * g.numel()), n
