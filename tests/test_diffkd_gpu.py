"""The engine's DiffKD head (kdfm.heads._diffkd_*, use_diffkd) against golden vectors from the
REFERENCE'S OWN DiffKDModule (tests/golden/make_golden_diffkd.py -> kd_diffkd.npz: 3 layer pairs,
B=2, T'=23; asr_train_diffm.py:326-394 with the training_step layer mean :795-800).

The head runs layer-batched beside version 1's heads (the lightest version); its loss is read from
its own accumulator, its parameter gradients from G["diffkd.*"], and its contribution to
d(loss)/d(student layer outputs) as the difference of two runs with and without DiffKD (same
inputs, same version heads).  f32 parity mode: loss rtol 1e-4, gradients max|diff| <= 1e-3 *
max|ref| + 1e-6.  bf16 mode (fused denoiser chain, the utterances replicated 40x so the stacked rows
take the benchmark's kernels; the per-layer means are unchanged, d/ds scales by 1/40): loss rtol 1e-2,
gradients relative Frobenius <= 3e-2."""
import os
from dataclasses import replace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_diffkd.npz")


def _run(cfg, P, Pfix, s_rows, t_rows, T, dev):
    from kdfm.heads import HeadsWorkspace, heads_backward, heads_forward
    G = {k: torch.zeros_like(v) for k, v in P.items()}
    ws = HeadsWorkspace(cfg, dev)
    acc = torch.zeros(5, device=dev)
    acc_d = torch.zeros(1, device=dev)
    seed = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx = heads_forward(cfg, P, s_rows, t_rows, T, ws, acc, seed=seed, save=True, Pfix=Pfix, acc_diffkd=acc_d)
    ds = torch.empty(s_rows.shape[0], cfg.d_student, device=dev)
    heads_backward(cfg, P, G, ctx, ws, ds, seed=seed)
    torch.cuda.synchronize()
    return acc_d.item(), G, ds


@pytest.mark.parametrize("math,copies,ltol,gtol,rn", [("f32", 1, 1e-4, 1e-3, None), ("bf16", 40, 1e-2, 1.0, 3e-2)])
def test_diffkd_matches_reference(math, copies, ltol, gtol, rn):
    from kdfm import kernels as K
    from kdfm.config import PARITY, head_specs
    from kdfm.store import init_uniform
    z = dict(np.load(GOLD, allow_pickle=False))
    L, B, T, steps = int(z["meta.L"]), int(z["meta.B"]), int(z["meta.T"]), int(z["meta.steps"])
    dev = torch.device("cuda")
    cfg = replace(PARITY, n_layers=L, math=math, version=1, use_diffkd=True, diffkd_steps=steps)
    s = torch.cat([torch.tensor(z[f"in.s{i}"]).repeat(copies, 1, 1).reshape(-1, 88) for i in range(L)])
    t = torch.cat([torch.tensor(z[f"in.t{i}"]).repeat(copies, 1, 1).reshape(-1, 176) for i in range(L)])
    s, t = s.contiguous().to(dev), t.contiguous().to(dev)
    P = {k: v.to(dev) for k, v in init_uniform(head_specs(cfg), 5).items()}
    for k in z:
        if k.startswith("param.") and not k.startswith("param.encoder."):
            P["diffkd." + k[6:]] = torch.tensor(z[k]).to(dev).contiguous()
    Pfix = {"diffkd." + k[6:]: torch.tensor(z[k]).to(dev).contiguous() for k in z if k.startswith("param.encoder.")}
    with K.mode(math, True):
        loss, G, ds = _run(cfg, P, Pfix, s, t, T, dev)
        _, _, ds0 = _run(replace(cfg, use_diffkd=False), P, Pfix, s, t, T, dev)
    ref = float(z["loss"])
    assert abs(loss - ref) <= ltol * abs(ref), (loss, ref)

    def close(a, b, what):
        a = a.detach().double().cpu()
        b = torch.as_tensor(b).double()
        err = (a - b).abs().max().item()
        scale = b.abs().max().item()
        assert err <= gtol * scale + 1e-6, f"{what}: max|diff| {err:.3e} vs max|ref| {scale:.3e}"
        if rn is not None:
            r = ((a - b).norm() / b.norm()).item()
            assert r <= rn, f"{what}: relative Frobenius error {r:.3e}"

    n = 0
    for k in z:
        if k.startswith("grad.") and not k.startswith("grad.s"):
            close(G["diffkd." + k[5:]], z[k], f"grad diffkd.{k[5:]}")
            n += 1
    assert n == 8   # decoder, proj, denoiser.{0,2} weights + biases; the encoder gets none
    dd = (ds - ds0).view(L, copies, B, T, 88)[:, 0] * copies
    for i in range(L):
        close(dd[i], z[f"grad.s{i}"], f"d/ds layer {i}")
