"""The engine's layer-batched KD heads (kdfm.heads: heads_forward / heads_backward, the fused
engine's path) for every model version 1-8 and kd_loss_type mse / l1, against the golden vectors
produced by the reference's own `_compute_v_losses_one_layer` (tests/golden/make_golden_versions.py,
asr_train_diffm.py:645-729).  fp32 parity mode (deterministic reductions); tolerances as
tests/test_versions_gpu.py: losses rtol 2e-4, d/ds max|diff| <= 2e-3 * max|ref|, per-parameter
gradient sum-of-squares rtol 5e-3 and sum within 5e-3 relative + 2e-3 * ||g|| * sqrt(numel).

Also pinned: the engine trains exactly the head modules whose reference gradients are non-zero
for the version (kdfm.config.head_modules; AdamW skips parameters without a gradient, so the rest
must stay out of the trained buffer)."""
import os
from dataclasses import replace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_heads_versions.npz")
KEYS = ("recon_loss", "kd_loss_pre", "fm_loss_pre", "kd_loss_post", "fm_loss_post")
CASES = [(v, "mse") for v in range(1, 9)] + [(1, "l1"), (3, "l1"), (8, "l1")]


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD, allow_pickle=False))


@pytest.mark.parametrize("version,kd", CASES)
def test_engine_heads_match_reference(gold, version, kd):
    from kdfm import kernels as K
    from kdfm.config import PARITY, head_specs
    from kdfm.heads import HeadsWorkspace, heads_backward, heads_forward
    cfg = replace(PARITY, n_layers=1, version=version, kd_loss_type=kd)
    dev = torch.device("cuda")
    B, T = int(gold["meta.B"]), int(gold["meta.T"])
    tag = f"v{version}{kd}"
    specs = dict(head_specs(cfg))
    # the trained set == the parameters the reference gives a gradient
    for k in gold:
        if k.startswith(f"{tag}.gsum."):
            name = k[len(f"{tag}.gsum."):]
            assert (name in specs) == (gold[k][1] != 0.0), (name, gold[k])
    P = {n: torch.tensor(gold["param." + n]).reshape(s).to(dev).contiguous() for n, s in specs.items()}
    G = {n: torch.zeros_like(p) for n, p in P.items()}
    s_rows = torch.tensor(gold["in.s"]).reshape(B * T, -1).contiguous().to(dev)
    t_rows = torch.tensor(gold["in.t"]).reshape(B * T, -1).contiguous().to(dev)
    eps = torch.tensor(gold["in.eps"]).transpose(1, 2).reshape(B * T, cfg.latent).contiguous().to(dev)
    with K.mode("f32", True):
        ws = HeadsWorkspace(cfg, dev)
        acc = torch.zeros(5, device=dev)
        seed = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx = heads_forward(cfg, P, s_rows, t_rows, T, ws, acc, seed=seed, eps=eps, save=True)
        ds = torch.empty(B * T, cfg.d_student, device=dev)
        heads_backward(cfg, P, G, ctx, ws, ds, seed=seed)
        torch.cuda.synchronize()
    got = acc.cpu().numpy()
    for i, k in enumerate(KEYS):
        np.testing.assert_allclose(float(got[i]), float(gold[f"{tag}.{k}"]), rtol=2e-4, atol=1e-6, err_msg=k)
    ref = gold[f"{tag}.grad.s"].reshape(B * T, -1)
    gs = ds.cpu().numpy()
    assert np.abs(gs - ref).max() <= 2e-3 * np.abs(ref).max() + 1e-6
    for n, g in G.items():
        r = gold[f"{tag}.gsum.{n}"]
        gg = g.double().cpu()
        s2 = float((gg ** 2).sum())
        np.testing.assert_allclose(s2, r[1], rtol=5e-3, err_msg=n)
        assert abs(float(gg.sum()) - r[0]) <= 5e-3 * abs(r[0]) + 2e-3 * np.sqrt(r[1] * g.numel()), n
