"""Fused SimpleDenoiser chain (csrc/denoise.hip: kdfm_denoise_chain_fwd / _bwd, bf16 MFMA with f32
state) and the CONV-mode bf16 weight gradient (kdfm_wgrad_bf16_conv) against float64 torch.

Reference: SimpleDenoiser.forward (asr_train_diffm.py:444-460) — S steps of x <- x - net(x)/S with
net = Conv1d(L,L,3,p=1) -> ReLU -> Conv1d(L,L,3,p=1) — over utterances of T frames, written with
torch.nn.functional.conv1d in float64 and differentiated by autograd (upstream gradient random).
T covers one window (29), the bench shape (401: two windows with halos) and many windows (1000);
a wrong halo would show as O(1) errors at the window seams.
Tolerances: relative Frobenius error <= 2e-2 for x_S, dL/dx_0 and every parameter gradient (bf16
operands, f32 accumulation over 2S convs); the weight-gradient kernel alone on exactly-bf16 operands
<= 1e-5 (f32 accumulation only).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _reference(z, W1, b1, W2, b2, gout, T, S):
    L = z.shape[1]
    U = z.shape[0] // T
    P = [t.double().clone().requires_grad_(True) for t in (z, W1, b1, W2, b2)]
    x = P[0].view(U, T, L).transpose(1, 2)
    for _ in range(S):
        x = x - F.conv1d(F.relu(F.conv1d(x, P[1], P[2], padding=1)), P[3], P[4], padding=1) / S
    out = x.transpose(1, 2).reshape(U * T, L)
    grads = torch.autograd.grad((out * gout.double()).sum(), P)
    return out.detach(), grads


@pytest.mark.parametrize("U,T", [(5, 29), (4, 401), (2, 1000)])
def test_denoise_chain_matches_float64(U, T):
    from kdfm import kernels as K
    L, S = 96, 9
    g = torch.Generator().manual_seed(T)
    n = U * T
    z = torch.randn(n, L, generator=g)
    bound = 1.0 / (3 * L) ** 0.5
    W1 = (torch.rand(L, L, 3, generator=g) * 2 - 1) * bound
    W2 = (torch.rand(L, L, 3, generator=g) * 2 - 1) * bound
    b1 = (torch.rand(L, generator=g) * 2 - 1) * bound
    b2 = (torch.rand(L, generator=g) * 2 - 1) * bound
    gout = torch.randn(n, L, generator=g)
    dev = "cuda"
    d = {k: v.to(dev) for k, v in dict(z=z, W1=W1, b1=b1, W2=W2, b2=b2, gout=gout).items()}
    X = torch.empty(S, n, L, device=dev, dtype=torch.bfloat16)
    A = torch.empty_like(X)
    out = torch.full((n, L), float("nan"), device=dev)
    K.denoise_chain_fwd(d["z"], d["W1"], d["b1"], d["W2"], d["b2"], X, A, out, T, S)
    GV = torch.empty_like(X)
    DA = torch.empty_like(X)
    gin = torch.full((n, L), float("nan"), device=dev)
    K.denoise_chain_bwd(d["gout"], A, d["W1"], d["W2"], GV, DA, gin, T, S)
    g1 = torch.zeros(L, 3 * L, device=dev)
    g2 = torch.zeros(L, 3 * L, device=dev)
    db1 = torch.zeros(L, device=dev)
    db2 = torch.zeros(L, device=dev)
    K.wgrad_bf16_conv(DA.view(S * n, L), X.view(S * n, L), g1, T, db=db1)
    K.wgrad_bf16_conv(GV.view(S * n, L), A.view(S * n, L), g2, T, alpha=-1.0 / S, db=db2)
    dW1 = torch.zeros(L, L, 3, device=dev)
    dW2 = torch.zeros(L, L, 3, device=dev)
    K.convw_grad(g1, dW1)
    K.convw_grad(g2, dW2)
    torch.cuda.synchronize()
    ref_out, (rz, rW1, rb1, rW2, rb2) = _reference(z, W1, b1, W2, b2, gout, T, S)
    assert torch.isfinite(out).all() and torch.isfinite(gin).all()
    for name, got, want in (("x_S", out, ref_out), ("dx0", gin, rz), ("dW1", dW1, rW1), ("db1", db1, rb1),
                            ("dW2", dW2, rW2), ("db2", db2, rb2)):
        assert _rel(got, want) <= 2e-2, (name, _rel(got, want))
    # the saved step-0 input is the bf16 image of z
    assert torch.equal(X[0].float(), z.to(dev).bfloat16().float())


def test_wgrad_bf16_conv_matches_float64():
    from kdfm import kernels as K
    g = torch.Generator().manual_seed(3)
    T, U, M, C = 37, 11, 96, 96
    rows = T * U
    dY = torch.randn(rows, M, generator=g).bfloat16()
    X = torch.randn(rows, C, generator=g).bfloat16()
    G = torch.zeros(M, 3 * C, device="cuda")
    db = torch.full((M,), 0.25, device="cuda")
    K.wgrad_bf16_conv(dY.cuda(), X.cuda(), G, T, db=db, alpha=0.5)
    torch.cuda.synchronize()
    xd = X.double().view(U, T, C)
    pad = F.pad(xd, (0, 0, 1, 1))                        # zero frame before/after each utterance
    cols = torch.cat([pad[:, tap:tap + T] for tap in range(3)], dim=2).view(rows, 3 * C)
    ref = 0.5 * dY.double().t() @ cols
    assert _rel(G, ref) <= 1e-5
    assert _rel(db - 0.25, 0.5 * dY.double().sum(0)) <= 1e-5
