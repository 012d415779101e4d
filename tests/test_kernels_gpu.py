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


@pytest.mark.parametrize("rows,d", [(1, 88), (63, 88), (12832, 88), (1000, 176), (77, 256), (130, 40),
                                    (1001, 512), (50, 768), (6432, 1024)])   # d % 256 == 0: the 16-byte-lane kernels
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
    if K.layernorm_bf16_ok(d):   # the bf16-output forward: the same values rounded to nearest even
        y16 = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
        m16, r16 = torch.empty_like(mean), torch.empty_like(rstd)
        K.layernorm_fwd(x, gam, bet, y16, m16, r16, 1e-5)
        torch.cuda.synchronize()
        assert torch.equal(y16, y.bfloat16()), "bf16 LN output differs from the rounded f32 output"
        assert torch.equal(m16, mean) and torch.equal(r16, rstd)


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


@pytest.mark.parametrize("batch_stats", [True, False])
@pytest.mark.parametrize("B,T,d,k", [(3, 401, 88, 31), (2, 70, 40, 15)])
def test_dwconv_bwd_bn_equals_separate(B, T, d, k, batch_stats):
    """kdfm_bn_silu_bwd_reduce + kdfm_dwconv_bwd_bn (the BN-SiLU backward's elementwise half applied on load)
    equal kdfm_bn_silu_bwd + kdfm_dwconv_bwd bit for bit (same formula, same operation order): dg, the folded
    depthwise weight / bias gradients and the BN affine gradients; red_next comes back zeroed."""
    K = _K()
    g = torch.Generator().manual_seed(B * T + d + k + 11)
    dz = torch.randn(B * T, d, generator=g).cuda()
    y = torch.randn(B * T, d, generator=g).cuda()
    gin = torch.randn(B * T, d, generator=g).cuda()
    w = torch.randn(d, k, generator=g).cuda()
    mean = torch.randn(d, generator=g).cuda() * 0.1
    rstd = torch.rand(d, generator=g).cuda() + 0.5
    gm = torch.randn(d, generator=g).cuda()
    bt = torch.randn(d, generator=g).cuda()
    # reference: separate BN-SiLU backward (memset + reduce + apply) then the depthwise backward
    red = torch.empty(2 * d, dtype=torch.float64, device="cuda")
    dy = torch.empty(B * T, d, device="cuda")
    dgm0, dbt0 = torch.zeros(d, device="cuda"), torch.zeros(d, device="cuda")
    K.bn_silu_bwd(dz, y, mean, rstd, gm, bt, red, dy, dgm0, dbt0, batch_stats=batch_stats)
    dg0 = torch.empty(B * T, d, device="cuda")
    dw0, db0 = torch.zeros(d, k, device="cuda"), torch.zeros(d, device="cuda")
    K.dwconv_bwd(dy, gin, w, dg0, dw0, db0, B, T, d, k)
    # fused
    red1 = torch.zeros(2 * d, dtype=torch.float64, device="cuda")
    red_next = torch.full((2 * d,), 7.0, dtype=torch.float64, device="cuda")
    dgm1, dbt1 = torch.zeros(d, device="cuda"), torch.zeros(d, device="cuda")
    K.bn_silu_bwd_reduce(dz, y, mean, rstd, gm, bt, red1)
    dg1 = torch.empty(B * T, d, device="cuda")
    ws = torch.empty(K.dwconv_bwd_ws(B, T, d, k), device="cuda")
    K.dwconv_bwd_bn(dz, y, mean, rstd, gm, bt, red1, red_next, dgm1, dbt1, batch_stats, gin, w, dg1, ws, B, T, d, k)
    dw1, db1 = torch.zeros(d, k, device="cuda"), torch.zeros(d, device="cuda")
    K.dwconv_bwd_fold(ws, dw1, db1, B, T, d, k)
    torch.cuda.synchronize()
    # the f64 sums are atomics (their order varies run to run): compare the affine grads to f32 rounding and
    # the rest to 1e-5 -- not bitwise even when the sums agree: the fused kernel forms dy on load with its
    # own FMA contraction of gamma rstd (dz silu' - m1 - xh m2), the separate BN-SiLU backward with another
    _close(dgm1, dgm0, rel=1e-6)
    _close(dbt1, dbt0, rel=1e-6)
    assert bool((red_next == 0).all())
    _close(dg1, dg0, rel=1e-5)
    _close(dw1, dw0, rel=1e-5)
    _close(db1, db0, rel=1e-5)


@pytest.mark.parametrize("B,T,d,k", [(3, 401, 88, 31), (2, 26, 88, 31), (2, 130, 176, 31), (2, 70, 40, 15),
                                     (2, 93, 1024, 9), (2, 65, 136, 31)])
def test_dwconv_bwd_channel_pairs_bitwise(B, T, d, k, monkeypatch):
    """The channel-pair depthwise backward (dwconv_bwd_p2_kernel: a lane owns 2 channels, 128 per workgroup,
    packed FMAs) equals the one-channel-per-lane kernel bit for bit -- dg, the weight / bias partials and
    their fold, plain and with the BN-SiLU backward applied on load (both schedules of the statistics),
    over one and several channel tiles and ragged frame tails."""
    K = _K()
    g = torch.Generator().manual_seed(B * T + d + k + 23)
    dz = torch.randn(B * T, d, generator=g).cuda()
    y = torch.randn(B * T, d, generator=g).cuda()
    gin = torch.randn(B * T, d, generator=g).cuda()
    w = torch.randn(d, k, generator=g).cuda()
    mean = torch.randn(d, generator=g).cuda() * 0.1
    rstd = torch.rand(d, generator=g).cuda() + 0.5
    gm = torch.randn(d, generator=g).cuda()
    bt = torch.randn(d, generator=g).cuda()
    red = torch.zeros(2 * d, dtype=torch.float64, device="cuda")
    K.bn_silu_bwd_reduce(dz, y, mean, rstd, gm, bt, red)
    outs = []
    for flag in ("0", "2"):
        monkeypatch.setenv("KDFM_DWC_P2", flag)
        dg = torch.empty(B * T, d, device="cuda")
        dw, db = torch.zeros(d, k, device="cuda"), torch.zeros(d, device="cuda")
        K.dwconv_bwd(dz, gin, w, dg, dw, db, B, T, d, k)
        res = [dg, dw, db]
        for bs in (True, False):
            red_next = torch.full((2 * d,), 7.0, dtype=torch.float64, device="cuda")
            dgm, dbt = torch.zeros(d, device="cuda"), torch.zeros(d, device="cuda")
            dg1 = torch.empty(B * T, d, device="cuda")
            ws = torch.full((K.dwconv_bwd_ws(B, T, d, k),), float("nan"), device="cuda")
            K.dwconv_bwd_bn(dz, y, mean, rstd, gm, bt, red, red_next, dgm, dbt, bs, gin, w, dg1, ws, B, T, d, k)
            dw1, db1 = torch.zeros(d, k, device="cuda"), torch.zeros(d, device="cuda")
            K.dwconv_bwd_fold(ws, dw1, db1, B, T, d, k)
            res += [dg1, dw1, db1, dgm, dbt, red_next]
        outs.append(res)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), f"output {i} differs"
    assert bool(torch.isfinite(outs[1][0]).all())


@pytest.mark.parametrize("B,T,d,k", [(3, 401, 88, 31), (2, 130, 176, 31), (2, 70, 40, 15), (2, 93, 1024, 9)])
def test_dwconv_fwd_channel_pairs(B, T, d, k, monkeypatch):
    """The channel-pair depthwise forward (dwconv_fwd_p2_kernel) writes bitwise the one-channel-per-lane kernel's y;
    its f64 BatchNorm sums (atomics: order varies) agree to 1e-12 relative."""
    K = _K()
    g = torch.Generator().manual_seed(B * T + d + k + 29)
    x = torch.randn(B * T, d, generator=g).cuda()
    w = torch.randn(d, k, generator=g).cuda()
    bias = torch.randn(d, generator=g).cuda()
    outs = []
    for flag in ("0", "2"):
        monkeypatch.setenv("KDFM_DWC_P2", flag)
        y = torch.empty(B * T, d, device="cuda")
        stats = torch.zeros(2 * d, dtype=torch.float64, device="cuda")
        K.dwconv_fwd(x, w, bias, y, stats, B, T, d, k)
        y2 = torch.empty(B * T, d, device="cuda")
        K.dwconv_fwd(x, w, None, y2, None, B, T, d, k)
        outs.append((y, stats, y2))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][2], outs[1][2])
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-12, atol=1e-9)
