"""The engine's layer-batched ver5 KD heads (kdfm.heads, HIP kernels) against the benchmark-shape
golden layer produced by the REFERENCE'S OWN classes (tests/golden/make_golden.py ->
kd_heads_ver5_b1t401.npz: one layer, B=1, T'=401 = 16.0 s of audio after 4x subsampling;
asr_train_diffm.py:400-497, 645-702, 1270-1427).

* f32 parity mode (deterministic reductions): the single utterance as the row batch.
  Tolerances: losses rtol 1e-4; every head-parameter gradient and d/ds max|diff| <= 1e-3 * max|ref| + 1e-6.
* bf16 throughput mode: the same utterance replicated 164x as the utterance axis of one layer
  (65 764 stacked rows: above the row counts at which kdfm_gemm switches to the row-streaming,
  weight-stationary, LDS-slab conv and wide-tile weight-gradient kernels the benchmark runs).  The
  per-layer means are unchanged by replication, so the losses and parameter gradients are the
  fixture's; d/ds of each copy is the fixture's / 164.  Tolerances (bf16 operands, f32 accumulate):
  losses rtol 1e-2; gradients relative Frobenius error <= 3e-2 and max|diff| <= 8e-2 * max|ref| + 1e-6
  (the NoiseAdapter gate gradient is a cancelling per-row reduction of bf16-rounded products).
"""
import os
from dataclasses import replace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_heads_ver5_b1t401.npz")


def _close(a, b, tol, what, rel_norm=None):
    a = a.detach().double().cpu()
    b = torch.as_tensor(b).double()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= tol * scale + 1e-6, f"{what}: max|diff| {err:.3e} vs max|ref| {scale:.3e}"
    if rel_norm is not None:
        rn = ((a - b).norm() / b.norm()).item()
        assert rn <= rel_norm, f"{what}: relative Frobenius error {rn:.3e}"


@pytest.mark.parametrize("math,copies,ltol,gtol,rn", [("f32", 1, 1e-4, 1e-3, None), ("bf16", 164, 1e-2, 8e-2, 3e-2)])
def test_heads_match_reference_layer(math, copies, ltol, gtol, rn):
    from kdfm import kernels as K
    from kdfm.config import PARITY
    from kdfm.heads import HeadsWorkspace, heads_backward, heads_forward
    gold = dict(np.load(GOLD, allow_pickle=False))
    cfg = replace(PARITY, n_layers=1, math=math)
    dev = torch.device("cuda")
    T = int(gold["meta.T"])
    s = torch.tensor(gold["in.s"])[0]            # (T, 88)  hook layout (B, T, C)
    t = torch.tensor(gold["in.t"])[0]            # (T, 176)
    eps = torch.tensor(gold["in.eps"])[0].t()    # (L, T) -> rows (T, L)
    n = copies * T
    s_rows = s.repeat(copies, 1).contiguous().to(dev)
    t_rows = t.repeat(copies, 1).contiguous().to(dev)
    eps_rows = eps.repeat(copies, 1).contiguous().to(dev)
    P, G = {}, {}
    for k, v in gold.items():
        if k.startswith("param.") and not k.startswith("param.fm_latent_2."):
            name = k[len("param."):]
            P[name] = torch.tensor(v).to(dev).contiguous()
            G[name] = torch.zeros_like(P[name])
    with K.mode(math, True):
        ws = HeadsWorkspace(cfg, dev)
        acc = torch.zeros(5, device=dev)   # recon, kd_pre, fm_pre, kd_post, fm_post
        seed = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx = heads_forward(cfg, P, s_rows, t_rows, T, ws, acc, seed=seed, eps=eps_rows, save=True)
        ds = torch.empty(n, cfg.d_student, device=dev)
        heads_backward(cfg, P, G, ctx, ws, ds, seed=seed)
        torch.cuda.synchronize()
    recon, kd_pre, fm_pre, kd_post, fm = acc.cpu().tolist()
    assert kd_pre == fm_pre == kd_post == 0.0   # ver5 adds only recon and fm_post
    assert abs(recon - float(gold["out.recon"])) <= ltol * abs(float(gold["out.recon"])), (recon, gold["out.recon"])
    assert abs(fm - float(gold["out.fm_post"])) <= ltol * abs(float(gold["out.fm_post"])), (fm, gold["out.fm_post"])
    checked = 0
    for name in P:
        _close(G[name], gold["grad." + name], gtol, f"grad {name} ({math})", rn)
        checked += 1
    assert checked == 22
    ref_ds = torch.tensor(gold["grad.in.s"])[0] / copies
    _close(ds.view(copies, T, -1)[0], ref_ds, gtol, f"d/ds ({math})", rn)
    _close(ds.view(copies, T, -1)[-1], ref_ds, gtol, f"d/ds last copy ({math})", rn)
