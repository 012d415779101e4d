"""Unit parity of the reduction-heavy backward kernels against torch fp32 autograd (the numerics
reference for a single floating-point op).  Tolerance: 1e-4 relative to the max |ref| (f32
accumulation-order differences only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _K():
    from kdfm import kernels as K
    return K


def _close(a, b, rel=1e-4):
    tol = rel * b.abs().max().item() + 1e-6
    err = (a - b).abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


@pytest.mark.parametrize("rows,d", [(1, 88), (63, 88), (12832, 88), (1000, 176), (77, 256), (130, 40)])
def test_layernorm_bwd(rows, d):
    K = _K()
    g = torch.Generator().manual_seed(rows + d)
    x = torch.randn(rows, d, generator=g).cuda()
    gam = torch.randn(d, generator=g).cuda()
    bet = torch.randn(d, generator=g).cuda()
    dy = torch.randn(rows, d, generator=g).cuda()
    dres = torch.randn(rows, d, generator=g).cuda()
    y = torch.empty_like(x)
    mean = torch.empty(rows, device="cuda")
    rstd = torch.empty(rows, device="cuda")
    K.layernorm_fwd(x, gam, bet, y, mean, rstd, 1e-5)
    xr, gr, br = (t.clone().requires_grad_() for t in (x, gam, bet))
    yr = torch.nn.functional.layer_norm(xr, (d,), gr, br, 1e-5)
    yr.backward(dy)
    dx = torch.empty_like(x)
    dg = torch.full((d,), 0.5, device="cuda")   # accumulates into existing grads
    db = torch.full((d,), -0.25, device="cuda")
    K.layernorm_bwd(dy, x, gam, mean, rstd, dx, dg, db, dres=dres)
    torch.cuda.synchronize()
    _close(y, yr.detach())
    _close(dx, xr.grad + dres)
    _close(dg - 0.5, gr.grad)
    _close(db + 0.25, br.grad)


@pytest.mark.parametrize("B,T,d,k", [(2, 26, 88, 31), (3, 401, 88, 31), (2, 130, 176, 31), (2, 70, 40, 15),
                                     (2, 50, 24, 7)])
def test_dwconv_bwd(B, T, d, k):
    K = _K()
    g = torch.Generator().manual_seed(B * T + d + k)
    x = torch.randn(B, T, d, generator=g).cuda()
    w = torch.randn(d, k, generator=g).cuda()
    bias = torch.randn(d, generator=g).cuda()
    dy = torch.randn(B, T, d, generator=g).cuda()
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, bias))
    yr = torch.nn.functional.conv1d(xr.transpose(1, 2), wr.unsqueeze(1), br, padding=(k - 1) // 2, groups=d)
    yr.transpose(1, 2).backward(dy)
    dx = torch.empty_like(x)
    dw = torch.zeros(d, k, device="cuda")
    db = torch.zeros(d, device="cuda")
    K.dwconv_bwd(dy, x, w, dx, dw, db, B, T, d, k)
    torch.cuda.synchronize()
    _close(dx, xr.grad)
    _close(dw, wr.grad)
    _close(db, br.grad)


@pytest.mark.parametrize("B,T,d,k", [(2, 26, 88, 31), (3, 401, 176, 31), (2, 70, 40, 15), (2, 50, 24, 7)])
def test_dwconv_fwd_stats(B, T, d, k):
    K = _K()
    g = torch.Generator().manual_seed(B * T + d + k + 1)
    x = torch.randn(B, T, d, generator=g).cuda()
    w = torch.randn(d, k, generator=g).cuda()
    bias = torch.randn(d, generator=g).cuda()
    y = torch.empty_like(x)
    stats = torch.zeros(2 * d, dtype=torch.float64, device="cuda")
    K.dwconv_fwd(x, w, bias, y, stats, B, T, d, k)
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv1d(x.transpose(1, 2), w.unsqueeze(1), bias, padding=(k - 1) // 2,
                                     groups=d).transpose(1, 2)
    _close(y, ref)
    r64 = ref.double().reshape(-1, d)
    torch.testing.assert_close(stats[:d], r64.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(stats[d:], (r64 * r64).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("B,T,d,k", [(3, 401, 88, 31), (2, 70, 40, 15)])
def test_dwconv_fwd_bn_finalize(B, T, d, k, det):
    """kdfm_dwconv_fwd_bn (the training BatchNorm finalize in the last workgroup of the depthwise conv) against
    float64 batch statistics and the running-statistics update; the sums and the counter are zero again after
    each call, so two layers' calls back to back on one pair agree with two separate references."""
    K = _K()
    from kdfm import _lib
    g = torch.Generator().manual_seed(B * T + d + k + 7)
    stats = torch.zeros(2 * d, dtype=torch.float64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    eps, mom = 1e-5, 0.1
    _lib.lib().kdfm_set_deterministic(1 if det else 0)
    try:
        for call in range(2):
            x = torch.randn(B, T, d, generator=g).cuda()
            w = torch.randn(d, k, generator=g).cuda()
            bias = torch.randn(d, generator=g).cuda()
            rm0 = torch.randn(d, generator=g).cuda()
            rv0 = torch.rand(d, generator=g).cuda() + 0.5
            rm, rv = rm0.clone(), rv0.clone()
            y = torch.empty_like(x)
            mean = torch.empty(d, device="cuda")
            rstd = torch.empty(d, device="cuda")
            K.dwconv_fwd_bn(x, w, bias, y, stats, cnt, rm, rv, mean, rstd, B, T, d, k, eps, mom)
            torch.cuda.synchronize()
            ref = torch.nn.functional.conv1d(x.transpose(1, 2), w.unsqueeze(1), bias, padding=(k - 1) // 2,
                                             groups=d).transpose(1, 2)
            _close(y, ref)
            r64 = ref.double().reshape(-1, d)
            m = r64.mean(0)
            var = r64.var(0, unbiased=False)
            torch.testing.assert_close(mean.double(), m, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(rstd.double(), 1.0 / torch.sqrt(var + eps), rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(rm.double(), (1 - mom) * rm0.double() + mom * m, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(rv.double(), (1 - mom) * rv0.double() + mom * r64.var(0, unbiased=True),
                                       rtol=1e-5, atol=1e-5)
            assert int(cnt.item()) == 0 and bool((stats == 0).all()), (call, cnt.item())
    finally:
        _lib.lib().kdfm_set_deterministic(0)
