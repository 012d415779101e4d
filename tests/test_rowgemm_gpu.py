"""Row-streaming d x d products (csrc/rowgemm.hip) against float64 torch and the unfused GPU path.

The products are ConformerLayer's attention linear_out (+ dropout + residual), the conv module's
BatchNorm + SiLU + pointwise_conv2 (+ dropout + residual) and their data gradients with the dropout
of the residual branch as prologue.  Tolerance: relative Frobenius <= 2e-2
against float64 (bf16 MFMA operands, f32 accumulation); the bf16 prologue copy must equal the bf16
rounding of the prologue output; dropout masks must match the standalone dropout kernel exactly.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("rows,d", [(12832, 88), (37, 88), (4010, 176)])
def test_rowgemm_resid_and_bnsilu(rows, d):
    from kdfm import kernels as K
    g = torch.Generator().manual_seed(rows + d)
    W = torch.randn(d, d, generator=g) / d ** 0.5
    b = 0.1 * torch.randn(d, generator=g)
    x = torch.randn(rows, d, generator=g)
    R = torch.randn(rows, d, generator=g)
    out = torch.empty(rows, d, device="cuda")
    xh = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    K.rowgemm(x.cuda(), K.rowgemm_img(W.cuda()), out, x_h=xh, epi=K.RG_EPI_RESID, bias=b.cuda(), R=R.cuda(), rscale=0.7)
    torch.cuda.synchronize()
    ref = R.double() + 0.7 * (x.double() @ W.double().t() + b.double())
    assert _rel(out - R.cuda(), ref - R.double()) <= 2e-2
    assert torch.equal(xh.cpu(), x.bfloat16())
    # BN-SiLU prologue
    mean = 0.1 * torch.randn(d, generator=g)
    rstd = 1.0 + 0.2 * torch.rand(d, generator=g)
    gam = 1.0 + 0.1 * torch.randn(d, generator=g)
    bet = 0.1 * torch.randn(d, generator=g)
    K.rowgemm(x.cuda(), K.rowgemm_img(W.cuda()), out, pro=K.RG_PRO_BNSILU,
              bn=(mean.cuda(), rstd.cuda(), gam.cuda(), bet.cuda()), x_h=xh, epi=K.RG_EPI_RESID, bias=b.cuda(),
              R=R.cuda(), rscale=1.0)
    torch.cuda.synchronize()
    z = torch.nn.functional.silu((x.double() - mean.double()) * rstd.double() * gam.double() + bet.double())
    ref = R.double() + (z @ W.double().t() + b.double())
    assert _rel(out - R.cuda(), ref - R.double()) <= 2e-2
    assert _rel(xh.float(), z) <= 5e-3


def test_rowgemm_dropout_prologue_data_gradient():
    from kdfm import kernels as K
    rows, d, p = 5003, 88, 0.1
    g = torch.Generator().manual_seed(9)
    W = (torch.randn(d, d, generator=g) / d ** 0.5).cuda()
    dy = torch.randn(rows, d, generator=g).cuda()
    seed = torch.tensor([987654321], dtype=torch.int64, device="cuda")
    dx = torch.empty(rows, d, device="cuda")
    dyh = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    K.rowgemm(dy, K.rowgemm_img(W, trans=True), dx, pro=K.RG_PRO_DROP, p_in=p, s_in=1.0, st_in=77, x_h=dyh, seed=seed)
    dd = torch.empty(rows, d, device="cuda")
    K.dropout(dy, dd, p, 1.0, seed, 77)
    torch.cuda.synchronize()
    assert torch.equal(dyh.float() == 0, dd == 0)
    assert _rel(dyh.float(), dd) <= 5e-3
    assert _rel(dx, dd.double() @ W.double()) <= 2e-2
    # forward dropout epilogue: same mask as the kdfm_gemm epilogue (K.linear, EPI_RESID | DROPOUT)
    from kdfm import _lib
    x = torch.randn(rows, d, generator=g).cuda()
    R = torch.randn(rows, d, generator=g).cuda()
    b = torch.zeros(d, device="cuda")
    o1 = torch.empty(rows, d, device="cuda")
    o2 = torch.empty(rows, d, device="cuda")
    K.rowgemm(x, K.rowgemm_img(W), o1, epi=K.RG_EPI_RESID, bias=b, R=R, rscale=1.0, p_out=p, st_out=78, seed=seed)
    with K.mode(math="bf16"):
        K.linear(x, W, b, o2, epi=_lib.EPI_RESID, R=R, rscale=1.0, dropout_p=p, seed=seed, rng_stream=78)
    torch.cuda.synchronize()
    assert torch.equal(o1 == R, o2 == R)
    assert _rel(o1 - R, o2 - R) <= 1e-2

