"""Fused FlowMatchingModule chain (csrc/fmchain.hip, bf16 MFMA with f32 state) and the bf16-operand
row-parallel weight gradient (kdfm_wgrad_bf16) against float64 torch references.

The chain is FlowMatchingModule.forward (asr_train_diffm.py:1368-1427; rectified schedule :852-856,
meta_encoder 'mlp', shape_transform 'linear') over rows, as kdfm/heads.py runs it; the reference
here is that recurrence written out in torch float64 and differentiated by autograd (same weights,
inputs, loss scale).  Tolerances: loss rtol 1e-2; every output, input gradient and parameter
gradient relative Frobenius error <= 2e-2 (bf16 operands, f32 accumulation over 8 steps);
kdfm_wgrad_bf16 on exactly-bf16 inputs: rel. Frobenius <= 1e-5 (f32 accumulation only).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_wgrad_bf16_matches_float64():
    from kdfm import kernels as K
    g = torch.Generator().manual_seed(0)
    rows, M, N = 5003, 96, 96
    dY = torch.randn(rows, M, generator=g).bfloat16()
    X = torch.randn(rows, N, generator=g).bfloat16()
    full = torch.zeros(M, 128)
    dW = full.cuda()[:, :N]            # row-strided destination (a meta_encoder.0 slice)
    db = torch.full((M,), 0.5).cuda()
    K.wgrad_bf16(dY.cuda(), X.cuda(), dW, db=db, alpha=0.75)
    torch.cuda.synchronize()
    ref = 0.75 * dY.double().t() @ X.double()
    assert _rel(dW, ref) <= 1e-5
    assert _rel(db - 0.5, 0.75 * dY.double().sum(0)) <= 1e-5


def _chain_ref(P, x0, zt, S, inv, gxs=None):
    """float64 FlowMatchingModule (rectified) over rows; returns loss, x_S and autograd grads."""
    L = x0.shape[1]
    P = {k: v.double().detach().clone().requires_grad_(True) for k, v in P.items()}
    x0 = x0.double().clone().requires_grad_(True)
    W1, b1, W2, b2 = P["W1"], P["b1"], P["W2"], P["b2"]
    te_w, te_b = P["te_w"], P["te_b"]
    x = x0
    v = None
    for i in range(S, 0, -1):
        t = torch.full((x.shape[0], 1), i / S, dtype=torch.float64)
        e = t @ te_w.t() + te_b
        a = torch.relu(torch.cat([x, e], 1) @ W1.t() + b1)
        v = a @ W2.t() + b2
        x = x - v / S
    nsx = x0 - v
    tr = nsx @ P["Wst"].t() + P["bst"]
    loss = inv * ((tr - zt.double()) ** 2).sum()
    total = loss + ((x * gxs.double()).sum() if gxs is not None else 0.0)
    grads = torch.autograd.grad(total, [x0] + list(P.values()))
    return loss.detach(), x.detach(), dict(zip(["x0"] + list(P), grads))


@pytest.mark.parametrize("with_out", [False, True])
def test_fused_fm_chain_matches_float64(with_out):
    from kdfm import kernels as K
    from kdfm.config import Ver5Config
    from kdfm.heads import HeadsWorkspace, _fm_backward, _fm_forward
    cfg = Ver5Config(math="bf16")
    L, E, S = cfg.latent, cfg.time_embed_dim, cfg.fm_steps
    n = 4133
    g = torch.Generator().manual_seed(1)
    pre = "fm_latent.fm."
    shapes = {"time_embed.weight": (E, 1), "time_embed.bias": (E,), "meta_encoder.0.weight": (L, L + E),
              "meta_encoder.0.bias": (L,), "meta_encoder.2.weight": (L, L), "meta_encoder.2.bias": (L,),
              "shape_transformation_function.weight": (L, L), "shape_transformation_function.bias": (L,)}
    P = {pre + k: ((torch.rand(s, generator=g) * 2 - 1) / (s[-1] ** 0.5 if len(s) > 1 else 3.0)) for k, s in shapes.items()}
    x0 = torch.randn(n, L, generator=g)
    zt = torch.randn(n, L, generator=g)
    gxs = torch.randn(n, L, generator=g) * 1e-3 if with_out else None
    inv = 1.0 / (n * L)
    dev = torch.device("cuda")
    Pd = {k: v.to(dev) for k, v in P.items()}
    Gd = {k: torch.zeros_like(v) for k, v in Pd.items()}
    with K.mode("bf16", False):
        ws = HeadsWorkspace(cfg, dev)
        acc = torch.zeros(1, device=dev)
        ctx, xs = _fm_forward(cfg, Pd, pre, ws, x0.to(dev), zt.to(dev), acc, inv, with_out, dev)
        assert ctx.get("fused"), "bf16 math must take the fused chain"
        gx0 = _fm_backward(cfg, Pd, Gd, ws, ctx, gxs.to(dev) if with_out else None, dev)
        torch.cuda.synchronize()
    ref = {"W1": P[pre + "meta_encoder.0.weight"], "b1": P[pre + "meta_encoder.0.bias"],
           "W2": P[pre + "meta_encoder.2.weight"], "b2": P[pre + "meta_encoder.2.bias"],
           "te_w": P[pre + "time_embed.weight"], "te_b": P[pre + "time_embed.bias"],
           "Wst": P[pre + "shape_transformation_function.weight"], "bst": P[pre + "shape_transformation_function.bias"]}
    loss, xS, grads = _chain_ref(ref, x0, zt, S, inv, gxs)
    assert abs(acc.item() - loss.item()) <= 1e-2 * abs(loss.item()), (acc.item(), loss.item())
    if with_out:
        assert _rel(xs, xS) <= 2e-2
    assert _rel(gx0, grads["x0"]) <= 2e-2
    names = {"W1": "meta_encoder.0.weight", "b1": "meta_encoder.0.bias", "W2": "meta_encoder.2.weight",
             "b2": "meta_encoder.2.bias", "te_w": "time_embed.weight", "te_b": "time_embed.bias",
             "Wst": "shape_transformation_function.weight", "bst": "shape_transformation_function.bias"}
    for k, nm in names.items():
        assert _rel(Gd[pre + nm], grads[k]) <= 2e-2, (nm, _rel(Gd[pre + nm], grads[k]))
