"""GPU numerics of the row-streaming GEMM paths (rowstream.hip) that kdfm_gemm selects for bf16
tall/narrow products and weight gradients.  Reference: torch fp32 matmul of the SAME bf16-rounded
operands, so the only difference is f32 accumulation order (tolerance 2e-3 of max |ref|)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from kdfm import kernels
    return kernels


def _bf(t):
    return t.to(torch.bfloat16).float()


def _close(out, ref, rel=2e-3):
    tol = rel * ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


def _conv3_ref(x, Wf, T):
    """out[r, o] = sum_{tap,c} Wf[o, tap*C + c] * x[r + tap - 1, c] within utterances of T rows"""
    M, C = x.shape
    U = M // T
    xs = x.view(U, T, C)
    pad = torch.nn.functional.pad(xs, (0, 0, 1, 1))
    taps = torch.cat([pad[:, t:t + T] for t in range(3)], dim=2)   # (U, T, 3C)
    return (taps.reshape(M, 3 * C) @ Wf.T)


@pytest.mark.parametrize("M,N,Kd", [(20000, 96, 96), (20011, 96, 88), (16384, 176, 96), (20000, 96, 176),
                                    (17000, 88, 88)])
def test_rowstream_linear(K, M, N, Kd):
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    R = torch.randn(M, N, device="cuda", generator=g)
    y = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, y, epi=_lib.EPI_RELU, math="bf16")
    h = _bf(x) @ _bf(W).T + b
    _close(y, torch.relu(h))
    K.linear(x, W, b, y, R=R, rscale=-0.125, epi=_lib.EPI_RESID, math="bf16")
    _close(y, R - 0.125 * h)
    # dx path (B contiguous along n) with the DRELU epilogue
    dy = torch.randn(M, N, device="cuda", generator=g)
    dx = torch.empty(M, Kd, device="cuda")
    aux = torch.randn(M, Kd, device="cuda", generator=g)
    K.linear_dx(dy, W, dx, epi=_lib.EPI_DRELU, aux=aux, alpha=-0.5, math="bf16")
    _close(dx, torch.where(aux > 0, -0.5 * (_bf(dy) @ _bf(W)), torch.zeros_like(aux)))


def test_rowstream_linear_mse(K):
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, Kd = 20000, 96, 96
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    tgt = torch.randn(M, N, device="cuda", generator=g)
    d = torch.empty(M, N, device="cuda")
    acc = torch.zeros(1, device="cuda")
    K.linear(x, W, b, d, R=tgt, rscale=2.0 / (M * N), mse=(acc, 1.0 / (M * N)), math="bf16")
    diff = _bf(x) @ _bf(W).T + b - tgt
    _close(d, diff * 2.0 / (M * N))
    ref = (diff ** 2).mean().item()
    assert abs(acc.item() - ref) <= 1e-4 * ref


@pytest.mark.parametrize("T,U", [(401, 50), (37, 500)])
def test_rowstream_conv3(K, T, U):
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(T)
    C = 96
    M = T * U
    x = torch.randn(M, C, device="cuda", generator=g)
    Wf = torch.randn(C, 3 * C, device="cuda", generator=g) * 0.05
    b = torch.randn(C, device="cuda", generator=g)
    R = torch.randn(M, C, device="cuda", generator=g)
    out = torch.empty(M, C, device="cuda")
    K.conv3(x, Wf, b, out, T, epi=_lib.EPI_RELU, math="bf16")
    ref = _conv3_ref(_bf(x), _bf(Wf), T) + b
    _close(out, torch.relu(ref))
    K.conv3(x, Wf, b, out, T, R=R, rscale=-1.0 / 9, math="bf16")
    _close(out, R - ref / 9)


@pytest.mark.parametrize("M,N,Kd,bias", [(20000, 96, 96, True), (12832, 88, 88, True), (12832, 352, 88, True),
                                         (12832, 88, 352, False), (12832, 264, 88, True), (205312 // 8, 176, 96, True),
                                         (8192, 96, 176, True)])
def test_rowstream_wgrad(K, M, N, Kd, bias):
    g = torch.Generator(device="cuda").manual_seed(N * 7 + Kd)
    dy = torch.randn(M, N, device="cuda", generator=g)
    x = torch.randn(M, Kd, device="cuda", generator=g)
    dW = torch.full((N, Kd), 0.25, device="cuda")
    db = torch.full((N,), -1.0, device="cuda") if bias else None
    K.linear_dw(dy, x, dW, alpha=-0.5, db=db, math="bf16")
    _close(dW - 0.25, -0.5 * (_bf(dy).T @ _bf(x)))
    if bias:
        _close(db + 1.0, -0.5 * _bf(dy).sum(0))


@pytest.mark.parametrize("T,U", [(401, 40), (64, 200)])
def test_rowstream_conv3_wgrad(K, T, U):
    g = torch.Generator(device="cuda").manual_seed(U)
    C = 96
    M = T * U
    dy = torch.randn(M, C, device="cuda", generator=g)
    x = torch.randn(M, C, device="cuda", generator=g)
    G = torch.zeros(C, 3 * C, device="cuda")
    db = torch.zeros(C, device="cuda")
    K.conv3_dw(dy, x, G, T, alpha=-1.0 / 9, db=db, math="bf16")
    xs = torch.nn.functional.pad(_bf(x).view(U, T, C), (0, 0, 1, 1))
    taps = torch.cat([xs[:, t:t + T] for t in range(3)], dim=2).reshape(M, 3 * C)
    _close(G, (-1.0 / 9) * (_bf(dy).T @ taps))
    _close(db, (-1.0 / 9) * _bf(dy).sum(0))
