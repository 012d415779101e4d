"""GPU numerics of the MFMA GEMM (kdfm_gemm) against plain torch fp32 on the same device."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from kdfm import kernels
    return kernels


def _tol(math):
    return (2e-5, 2e-5) if math == "f32" else (3e-2, 3e-2)


@pytest.mark.parametrize("math", ["f32", "bf16"])
@pytest.mark.parametrize("M,N,Kd", [(12832, 88, 352), (100, 129, 88), (65, 33, 44), (1, 1, 1), (300, 704, 176)])
def test_linear_fwd_dx_dw(K, math, M, N, Kd):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    y = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, y, math=math)
    ref = x @ W.T + b
    rt, at = _tol(math)
    torch.testing.assert_close(y, ref, rtol=rt, atol=at * ref.abs().max().item())
    dy = torch.randn(M, N, device="cuda", generator=g)
    dx = torch.empty(M, Kd, device="cuda")
    K.linear_dx(dy, W, dx, math=math)
    ref = dy @ W
    torch.testing.assert_close(dx, ref, rtol=rt, atol=at * ref.abs().max().item())
    dW = torch.zeros(N, Kd, device="cuda")
    K.linear_dw(dy, x, dW, math=math)
    ref = dy.T @ x
    torch.testing.assert_close(dW, ref, rtol=rt, atol=at * ref.abs().max().item() + 1e-5)


@pytest.mark.parametrize("math", ["f32", "bf16"])
def test_epilogues(K, math):
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(1)
    M, N, Kd = 500, 176, 88
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.2
    b = torch.randn(N, device="cuda", generator=g)
    R = torch.randn(M, N, device="cuda", generator=g)
    pre = torch.empty(M, N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, out, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE | _lib.EPI_RESID, R=R, rscale=0.5,
                 Cpre=pre, math=math)
    h = x @ W.T + b
    rt, at = _tol(math)
    torch.testing.assert_close(pre, h, rtol=rt, atol=at * h.abs().max().item())
    ref = R + 0.5 * torch.nn.functional.silu(h)
    torch.testing.assert_close(out, ref, rtol=rt, atol=at * ref.abs().max().item())


def test_conv3_mode(K):
    """Conv1d(k=3, pad=1) over frames via the CONV A-operand, f32 parity mode."""
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(2)
    Bn, T, Cc = 3, 37, 96
    x = torch.randn(Bn, T, Cc, device="cuda", generator=g)
    W = torch.randn(Cc, Cc, 3, device="cuda", generator=g) * 0.1  # Conv1d weight (out, in, k)
    b = torch.randn(Cc, device="cuda", generator=g)
    Wk = W.permute(0, 2, 1).contiguous()  # (out, tap, in) -> B(k=tap*C+c, n=o) = Wk[o, k]
    out = torch.empty(Bn * T, Cc, device="cuda")
    K.gemm(x, Wk, out, Bn * T, Cc, 3 * Cc, Cc, 1, 1, 3 * Cc, Cc, 1, amode=_lib.LD_CONV, bmode=_lib.LD_KC,
           epi=_lib.EPI_BIAS, bias=b, conv=(3, 1, Cc, T), math="f32")
    ref = torch.nn.functional.conv1d(x.transpose(1, 2), W, b, padding=1).transpose(1, 2).reshape(Bn * T, Cc)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("kind", ["silu", "resid"])
def test_bf16_dropout_epilogues_match_f32_path(kind):
    """The compile-time FFN epilogues of the bf16 GEMM (SiLU+dropout+STORE_PRE, dropout+residual)
    against the generic f32 GEMM followed by the standalone dropout kernel with the same counter
    RNG: identical drop pattern, values within bf16 tolerance."""
    from kdfm import _lib
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(7)
    M, Kd, N = 12832, 88, 352 if kind == "silu" else 88
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    R = torch.randn(M, N, device="cuda", generator=g)
    seed = torch.tensor([12345], dtype=torch.int64, device="cuda")
    p = 0.1
    y = torch.empty(M, N, device="cuda")
    pre = torch.empty(M, N, device="cuda")
    ref_pre = torch.empty(M, N, device="cuda")
    if kind == "silu":
        K.linear(x, W, b, y, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE, Cpre=pre, dropout_p=p, seed=seed,
                 rng_stream=5, math="bf16")
        K.linear(x, W, b, ref_pre, math="f32")
        act = torch.nn.functional.silu(ref_pre)
    else:
        K.linear(x, W, b, y, epi=_lib.EPI_RESID, R=R, rscale=0.5, dropout_p=p, seed=seed, rng_stream=5,
                 math="bf16")
        K.linear(x, W, b, ref_pre, math="f32")
        act = ref_pre.clone()
    ref = torch.empty_like(act)
    K.dropout(act.contiguous(), ref, p, 1.0, seed, 5)
    if kind == "resid":
        ref = R + 0.5 * ref
        kept = (y - R).abs() > 0
        want_kept = (ref - R).abs() > 0
    else:
        kept = y != 0
        want_kept = ref != 0
        torch.testing.assert_close(pre, ref_pre, rtol=2e-2, atol=2e-2)
    assert torch.equal(kept, want_kept)
    torch.testing.assert_close(y, ref, rtol=2e-2, atol=3e-2)
