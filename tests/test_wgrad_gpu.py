"""The row-parallel weight-gradient kernel (csrc/wgrad.hip, kdfm_gemm route "wgrad_rows") against
torch fp32 on the same device: every wave-tile instance, the implicit ones column (bias gradient),
alpha, accumulation into a non-zero gradient, rows that are not a multiple of the 32-row step,
multi-slice wide outputs, and the Conv1d(k=3) CONV mode with utterance boundaries.  bf16 operands,
f32 accumulation: max|diff| <= 2e-2 * max|ref|.  Also: bitwise reproducible (ordered fold)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # rows, M (dY cols), N (X cols), bias
    (12832, 88, 352, True), (12832, 352, 88, True), (12832, 264, 88, True), (12832, 176, 88, True),
    (12832, 88, 88, True), (12832, 88, 1760, False), (25600, 88, 792, True), (205312 // 8, 96, 96, True),
    (205312 // 8, 96, 176, True), (205312 // 8, 176, 96, True), (4097, 96, 88, True), (2049, 128, 20, True),
]


def _route():
    from kdfm import _lib, kernels as K
    return K.ROUTES.get(int(_lib.lib().kdfm_gemm_last_route()))


@pytest.mark.parametrize("R,M,N,bias", SHAPES)
def test_linear_dw_rows(R, M, N, bias):
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(R + M + N)
    dy = torch.randn(R, M, device="cuda", generator=g)
    x = torch.randn(R, N, device="cuda", generator=g)
    dW0 = torch.randn(M, N, device="cuda", generator=g)
    db0 = torch.randn(M, device="cuda", generator=g)
    dW, db = dW0.clone(), db0.clone()
    alpha = -0.37
    with K.mode("bf16"):
        K.linear_dw(dy, x, dW, alpha=alpha, db=db if bias else None)
    assert _route() == "wgrad_rows"
    ref = dW0 + alpha * (dy.double().T @ x.double()).float()
    scale = (dy.double().T @ x.double()).abs().max().item() * abs(alpha)
    assert (dW - ref).abs().max().item() <= 2e-2 * scale
    if bias:
        rb = db0 + alpha * dy.double().sum(0).float()
        assert (db - rb).abs().max().item() <= 2e-2 * dy.double().sum(0).abs().max().item() * abs(alpha) + 1e-4
    else:
        assert torch.equal(db, db0)
    # ordered fold: a second identical call adds bitwise the same increment
    dW2 = dW0.clone()
    with K.mode("bf16"):
        K.linear_dw(dy, x, dW2, alpha=alpha, db=None)
        dW3 = dW0.clone()
        K.linear_dw(dy, x, dW3, alpha=alpha, db=None)
    assert torch.equal(dW2, dW3)


@pytest.mark.parametrize("B,T", [(64, 401), (37, 123)])
def test_conv3_dw_rows(B, T):
    """SimpleDenoiser Conv1d(96, 96, 3, padding=1) weight gradient over utterances of T frames."""
    from kdfm import kernels as K
    C = 96
    g = torch.Generator(device="cuda").manual_seed(B * T)
    x = torch.randn(B, T, C, device="cuda", generator=g)
    dy = torch.randn(B, T, C, device="cuda", generator=g)
    G = torch.zeros(C, 3 * C, device="cuda")
    db = torch.zeros(C, device="cuda")
    with K.mode("bf16"):
        K.conv3_dw(dy.view(B * T, C), x.view(B * T, C), G, T, alpha=0.5, db=db)
    assert _route() == "wgrad_rows"
    xr = x.double().transpose(1, 2).requires_grad_(True)
    W = torch.zeros(C, C, 3, dtype=torch.float64, device="cuda", requires_grad=True)
    bb = torch.zeros(C, dtype=torch.float64, device="cuda", requires_grad=True)
    out = torch.nn.functional.conv1d(xr, W, bb, padding=1)
    gW, gb = torch.autograd.grad(out, [W, bb], dy.double().transpose(1, 2))
    ref = 0.5 * gW.permute(0, 2, 1).reshape(C, 3 * C)   # GEMM layout G[o, tap*C + c]
    assert (G.double() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert (db.double() - 0.5 * gb).abs().max().item() <= 2e-2 * (0.5 * gb).abs().max().item()
