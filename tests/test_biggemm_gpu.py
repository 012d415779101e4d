"""The large-tile bf16 GEMM (csrc/biggemm.hip, kdfm_gemm_big) behind kernels.linear / linear_dx / linear_dw for the
wide layer products (d_model >= 512: Conformer-large, FastConformer-XL -- BASELINE.json configs[3] / [4]; the
Linear layers of conformer_encoder.py:450-472 at fast-conformer_ctc_bpe.yaml:29's widths).

Reference: float64 torch matmul of the bf16-ROUNDED operands (the kernel's MFMAs take bf16 operands exactly and
accumulate in f32), tolerance 2e-6 of sum_k |a_k b_k| per element -- K * 2^-24 relative f32 accumulation error at the
largest K here (4096) is ~2.4e-4 worst case, the observed error is orders below that; the bound is stated per
element against the absolute-product sum, which is what f32 accumulation error scales with.  Epilogues (bias, SiLU,
dropout with STORE_PRE, residual, dSiLU with dropout) against the same formula applied in float64 with the kernel's
own dropout mask read back from the output's zero pattern cross-checked against the generic kdfm_gemm route's mask
(same counter-RNG index).  Shapes cover partial row / column tiles, all three tile shapes, a reduction-row tail (TN),
bf16 in-place operands and bf16 output.  Deterministic: a second run is bitwise equal.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _all_sizes(monkeypatch):
    """every product here takes the large-tile route, whatever its size (the production floor is M N K >= 2^31)"""
    from kdfm import kernels as K
    monkeypatch.setattr(K, "_BIG_MIN_WORK", 0.0)


def _K():
    from kdfm import kernels as K
    K.set_math("bf16")
    return K


def _rb(t):
    return t.bfloat16().double()


def _check(got, ref, absprod, tol=2e-6):
    err = (got.double() - ref).abs()
    bound = tol * absprod + 1e-30
    worst = float((err / bound).max())
    assert worst <= 1.0, f"max err / bound = {worst:.3g}"


@pytest.mark.parametrize("M,N,K_", [(6432, 4096, 1024), (6432, 1024, 4096), (3001, 640, 512), (1111, 1536, 768)])
def test_linear_forward_plain_and_bias(M, N, K_):
    K = _K()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(M + N)
    x = torch.randn(M, K_, device=dev, generator=g)
    W = torch.randn(N, K_, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    assert K.big_ok(M, N, K_, 0)
    y = torch.empty(M, N, device=dev)
    K.linear(x, W, b, y)
    import kdfm._lib as L
    assert K.ROUTES[int(L.lib().kdfm_gemm_last_route())] == "big"
    ref = _rb(x) @ _rb(W).t() + b.double()
    _check(y, ref, _rb(x).abs() @ _rb(W).abs().t())
    y2 = torch.empty_like(y)
    K.linear(x, W, b, y2)
    assert torch.equal(y, y2), "not deterministic"


@pytest.mark.parametrize("M,N,K_", [(5000, 1024, 96), (4100, 96, 1024), (3000, 256, 200), (2000, 136, 264)])
def test_wide_mode_narrow_products_and_k_tails(M, N, K_, monkeypatch):
    """The wide-model mode (set_wide: FastConformer-XL) sends products with a dimension in [64, 512) to the large-tile
    route: the distillation heads' d -> 1024 / 1024 -> d projections (K or N = 96), the 256-channel pointwise convs;
    K % 64 != 0 exercises the k-contiguous images' zeroed tail step (forward NT over K, data gradient NN over N)."""
    K = _K()
    import kdfm._lib as L
    monkeypatch.setattr(K._State, "wide", True)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(M + 7 * N + K_)
    x = torch.randn(M, K_, device=dev, generator=g)
    W = torch.randn(N, K_, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    assert K.big_ok(M, N, K_, L.BIG_NT)
    y = torch.empty(M, N, device=dev)
    K.linear(x, W, b, y)
    assert K.ROUTES[int(L.lib().kdfm_gemm_last_route())] == "big"
    _check(y, _rb(x) @ _rb(W).t() + b.double(), _rb(x).abs() @ _rb(W).abs().t() + b.double().abs())
    dy = torch.randn(M, N, device=dev, generator=g)
    dx = torch.empty(M, K_, device=dev)
    if K.big_ok(M, K_, N, L.BIG_NN):
        K.linear_dx(dy, W, dx)
        assert K.ROUTES[int(L.lib().kdfm_gemm_last_route())] == "big"
        _check(dx, _rb(dy) @ _rb(W), _rb(dy).abs() @ _rb(W).abs())
    monkeypatch.setattr(K._State, "wide", False)
    assert not K.big_ok(M, N, K_, L.BIG_NT), "narrow products leave the large-tile route outside the wide mode"


def test_linear_silu_dropout_store_pre_bf16_out_and_residual():
    K = _K()
    import kdfm._lib as L
    dev = "cuda"
    M, d, ff = 4111, 512, 2048
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(M, d, device=dev, generator=g)
    W1 = torch.randn(ff, d, device=dev, generator=g) * 0.05
    b1 = torch.randn(ff, device=dev, generator=g) * 0.1
    W2 = torch.randn(d, ff, device=dev, generator=g) * 0.03
    b2 = torch.randn(d, device=dev, generator=g) * 0.1
    seed = torch.tensor([1234567], dtype=torch.int64, device=dev)
    # up-projection: bias + SiLU + dropout, pre-activation stored (f32), activation out in bf16
    a16 = torch.empty(M, ff, device=dev, dtype=torch.bfloat16)
    h = torch.empty(M, ff, device=dev)
    K.linear(x, W1, b1, a16, epi=L.EPI_SILU | L.EPI_STORE_PRE, Cpre=h, dropout_p=0.1, seed=seed, rng_stream=77)
    pre = _rb(x) @ _rb(W1).t() + b1.double()
    _check(h, pre, _rb(x).abs() @ _rb(W1).abs().t() + b1.double().abs())
    # the generic route with the same flags draws the same dropout mask
    K._BIG = False
    try:
        a_gen = torch.empty(M, ff, device=dev)
        K.linear(x, W1, b1, a_gen, epi=L.EPI_SILU, dropout_p=0.1, seed=seed, rng_stream=77)
    finally:
        K._BIG = True
    keep = a_gen != 0
    assert torch.equal(keep, a16 != 0), "dropout mask differs from the generic route's"
    silu = h.double() * torch.sigmoid(h.double())
    ref_a = torch.where(keep, silu / 0.9, torch.zeros_like(silu))
    assert torch.allclose(a16.double(), ref_a.bfloat16().double(), rtol=1e-2, atol=1e-3)
    frac = 1.0 - keep.double().mean().item()
    assert 0.09 < frac < 0.11
    # down-projection from the bf16 activation in place: bias + dropout + 0.5 * residual
    out = torch.empty(M, d, device=dev)
    K.linear(a16, W2, b2, out, epi=L.EPI_RESID, R=x, rscale=0.5, dropout_p=0.1, seed=seed, rng_stream=78)
    lin = a16.double() @ _rb(W2).t() + b2.double()
    keep2 = (out - x) != 0
    ref = x.double() + 0.5 * torch.where(keep2, lin / 0.9, torch.zeros_like(lin))
    _check(out - x, ref - x.double(), 0.5 / 0.9 * (a16.double().abs() @ _rb(W2).abs().t() + b2.double().abs()), 1e-5)


def test_linear_dx_dsilu_dropout_bf16_out():
    K = _K()
    import kdfm._lib as L
    dev = "cuda"
    M, d, ff = 6432, 1024, 4096
    g = torch.Generator(device=dev).manual_seed(4)
    dy = torch.randn(M, d, device=dev, generator=g)
    W2 = torch.randn(d, ff, device=dev, generator=g) * 0.03
    h = torch.randn(M, ff, device=dev, generator=g)
    seed = torch.tensor([99], dtype=torch.int64, device=dev)
    assert K.big_ok(M, ff, d, L.BIG_NN)
    dh = torch.empty(M, ff, device=dev)
    K.linear_dx(dy, W2, dh, epi=L.EPI_DSILU, aux=h, dropout_p=0.1, seed=seed, rng_stream=5)
    K._BIG = False
    try:
        dh_gen = torch.empty(M, ff, device=dev)
        K.linear_dx(dy, W2, dh_gen, epi=L.EPI_DSILU, aux=h, dropout_p=0.1, seed=seed, rng_stream=5)
    finally:
        K._BIG = True
    keep = dh_gen != 0
    assert torch.equal(keep, dh != 0), "dropout mask differs from the generic route's"
    s = torch.sigmoid(h.double())
    dsilu = s * (1 + h.double() * (1 - s))
    prod = _rb(dy) @ _rb(W2)
    ref = torch.where(keep, prod / 0.9, torch.zeros_like(prod)) * dsilu
    # the f32 product's accumulation error times |silu'|, plus silu' itself from v_exp_f32 / v_rcp_f32 (a few ulp,
    # absolute: the derivative crosses zero at h ~ -1.28, where a relative bound alone would demand exactness)
    _check(dh, ref, (_rb(dy).abs() @ _rb(W2).abs()) / 0.9 * (dsilu.abs() + 2.0), 4e-6)
    dh16 = torch.empty(M, ff, device=dev, dtype=torch.bfloat16)
    K.linear_dx(dy, W2, dh16, epi=L.EPI_DSILU, aux=h, dropout_p=0.1, seed=seed, rng_stream=5)
    assert torch.equal(dh16, dh.bfloat16()), "bf16 output must be the f32 result rounded"


@pytest.mark.parametrize("M,N,K_", [(6432, 1024, 4096), (6432, 4096, 1024), (3001, 512, 768)])
def test_linear_dx_plain(M, N, K_):
    """dx[M, K_] = dy[M, N] W[N, K_]"""
    K = _K()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(7)
    dy = torch.randn(M, N, device=dev, generator=g)
    W = torch.randn(N, K_, device=dev, generator=g) * 0.05
    dx = torch.empty(M, K_, device=dev)
    K.linear_dx(dy, W, dx)
    _check(dx, _rb(dy) @ _rb(W), _rb(dy).abs() @ _rb(W).abs())


@pytest.mark.parametrize("M,N,K_,bias", [(6432, 4096, 1024, True), (6432, 1024, 4096, True), (6432, 1024, 1024, False),
                                        (3001, 640, 512, True)])
def test_linear_dw_accumulate_and_bias(M, N, K_, bias):
    """dW[N, K_] += alpha dy^T x, db[N] += alpha colsum(dy); rows M not a multiple of 64 (k-major tail)"""
    K = _K()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(11)
    dy = torch.randn(M, N, device=dev, generator=g)
    x = torch.randn(M, K_, device=dev, generator=g)
    dW0 = torch.randn(N, K_, device=dev, generator=g)
    db0 = torch.randn(N, device=dev, generator=g)
    dW, db = dW0.clone(), db0.clone()
    K.linear_dw(dy, x, dW, db=db if bias else None, alpha=0.5)
    ref = dW0.double() + 0.5 * (_rb(dy).t() @ _rb(x))
    _check(dW - dW0, ref - dW0.double(), 0.5 * (_rb(dy).abs().t() @ _rb(x).abs()))
    if bias:
        rdb = db0.double() + 0.5 * _rb(dy).sum(0)
        _check(db - db0, rdb - db0.double(), 0.5 * _rb(dy).abs().sum(0))
    dW2 = dW0.clone()
    db2 = db0.clone()
    K.linear_dw(dy, x, dW2, db=db2 if bias else None, alpha=0.5)
    assert torch.equal(dW, dW2) and torch.equal(db, db2), "not deterministic"


@pytest.mark.parametrize("tile", ["0", "1", "2"])
def test_every_tile_shape(tile, monkeypatch):
    """each of the three tile shapes (KDFM_BIG_TILE forces one) on each layout"""
    monkeypatch.setenv("KDFM_BIG_TILE", tile)
    K = _K()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(21)
    M, N, K_ = 2100, 768, 1024
    x = torch.randn(M, K_, device=dev, generator=g)
    W = torch.randn(N, K_, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    y = torch.empty(M, N, device=dev)
    K.linear(x, W, b, y)
    _check(y, _rb(x) @ _rb(W).t() + b.double(), _rb(x).abs() @ _rb(W).abs().t() + b.double().abs())
    dx = torch.empty(M, K_, device=dev)
    K.linear_dx(y, W, dx)
    _check(dx, _rb(y) @ _rb(W), _rb(y).abs() @ _rb(W).abs())
    dW = torch.zeros(N, K_, device=dev)
    db = torch.zeros(N, device=dev)
    K.linear_dw(y, x, dW, db=db)
    _check(dW, _rb(y).t() @ _rb(x), _rb(y).abs().t() @ _rb(x).abs())
    _check(db, _rb(y).sum(0), _rb(y).abs().sum(0))


# ---- fp8 e4m3 instance, MX block scaling (Ver5Config.linear_fp8; BASELINE.json configs[4]) ----

def _mx(t):
    """torch restatement of kdfm_fp8_quant_mx along the last dim: per 32-block e = ceil(log2(amax / 448)) (amax = 0:
    -127), q = e4m3fn(x 2^-e); returns (q as e4m3fn, e per block as int), float64 math"""
    x = t.double().reshape(t.shape[0], -1, 32)
    amax = x.abs().max(2, keepdim=True).values
    e = torch.ceil(torch.log2(amax.clamp_min(1e-300) / 448.0))
    e = torch.where(amax > 0, e, torch.full_like(e, -127.0)).clamp(-127, 127)
    q = (x / torch.pow(2.0, e)).float().to(torch.float8_e4m3fn).reshape(t.shape)
    return q, e.squeeze(2).long()


def _deq(q, e):
    return (q.double().reshape(q.shape[0], -1, 32) * torch.pow(2.0, e.double()).unsqueeze(2)).reshape(q.shape)


def _stage_major(e):
    """[R][K/32] block exponents -> the kernel's stage-major scale bytes [(K/128)][R][4]"""
    R, nb = e.shape
    return (e + 127).to(torch.uint8).view(R, nb // 4, 4).permute(1, 0, 2).contiguous().view(-1)


def test_fp8_mx_quantisation_matches_torch():
    K = _K()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(31)
    x = torch.randn(1000, 768, device=dev, generator=g) * 3
    x[5, 64:96] = 0.0                       # an all-zero block
    x[7, 0] = 1e4                           # an outlier block
    W = torch.randn(512, 768, device=dev, generator=g) * 0.02
    (xa, lx, xs), (wa, lw, ws_) = K._fp8_operands([(x, False), (W, True)])
    torch.cuda.synchronize()
    buf = K.scratch(x.device, 1).view(torch.uint8)
    base = buf.data_ptr()
    xq = buf[xa - base: xa - base + 1000 * lx].view(1000, lx)[:, :768]
    wq = buf[wa - base: wa - base + 768 * lw].view(768, lw)[:, :512]
    xsb = buf[xs - base: xs - base + 1000 * 768 // 32]
    wsb = buf[ws_ - base: ws_ - base + 768 * 512 // 32]
    rq, re = _mx(x)
    rwq, rwe = _mx(W.t().contiguous())
    assert torch.equal(xsb, _stage_major(re)), "row-major block scales differ"
    assert torch.equal(xq, rq.view(torch.uint8)), "row-major MX quantisation differs from torch e4m3fn"
    assert torch.equal(wsb, _stage_major(rwe)), "transposed block scales differ"
    assert torch.equal(wq, rwq.view(torch.uint8)), "transposed MX quantisation differs"
    # bf16 sources (the large-tile route's activations): the row-tiled kernel (16-byte rows) and the
    # 8-lanes-per-block kernel (a row stride that is not a multiple of 8 elements) give the same bytes
    for cols_ld in (768, 772):
        xb = torch.zeros(1000, cols_ld, device=dev, dtype=torch.bfloat16)
        xb[:, :768] = x.bfloat16()
        xv = xb[:, :768]
        ((ba, lb, bs),) = K._fp8_operands([(xv, False)])
        torch.cuda.synchronize()
        buf = K.scratch(x.device, 1).view(torch.uint8)
        base = buf.data_ptr()
        bq = buf[ba - base: ba - base + 1000 * lb].view(1000, lb)[:, :768]
        bsb = buf[bs - base: bs - base + 1000 * 768 // 32]
        rbq, rbe = _mx(xv.float())
        assert torch.equal(bsb, _stage_major(rbe)), f"bf16 block scales differ (ld {cols_ld})"
        assert torch.equal(bq, rbq.view(torch.uint8)), f"bf16 MX quantisation differs (ld {cols_ld})"


@pytest.mark.parametrize("M,N,K_", [(6432, 4096, 1024), (3000, 640, 512)])
def test_fp8_linear_forward_and_dx(M, N, K_, monkeypatch):
    K = _K()
    monkeypatch.setattr(K._State, "fp8", True)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(M)
    x = torch.randn(M, K_, device=dev, generator=g)
    W = torch.randn(N, K_, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    n = {"fp8": 0}
    orig = K.call

    def call(name, *a):
        n["fp8"] += name == "kdfm_gemm_big_fp8"
        return orig(name, *a)
    monkeypatch.setattr(K, "call", call)
    y = torch.empty(M, N, device=dev)
    K.linear(x, W, b, y)
    xd, wd = _deq(*_mx(x)), _deq(*_mx(W))
    # the block-scaled fp8 MFMA's accumulation is not an f32 fmaf chain over k: measured up to ~1.1e-5 of the
    # absolute-product sum (profiles/r06), hence 2e-5 (the e4m3 rounding itself is ~6e-2 relative)
    _check(y, xd @ wd.t() + b.double(), xd.abs() @ wd.abs().t() + b.double().abs(), 2e-5)
    dy = torch.randn(M, N, device=dev, generator=g)
    dxo = torch.empty(M, K_, device=dev)
    K.linear_dx(dy, W, dxo)
    dd, wtd = _deq(*_mx(dy)), _deq(*_mx(W.t().contiguous()))
    _check(dxo, dd @ wtd.t(), dd.abs() @ wtd.abs().t(), 2e-5)
    assert n["fp8"] == 2, n
    y2 = torch.empty_like(y)
    K.linear(x, W, b, y2)
    assert torch.equal(y, y2), "not deterministic"


def test_fp8_silu_dropout_epilogue_bf16_out(monkeypatch):
    K = _K()
    import kdfm._lib as L
    monkeypatch.setattr(K._State, "fp8", True)
    dev = "cuda"
    M, d, ff = 2048, 512, 2048
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(M, d, device=dev, generator=g)
    W1 = torch.randn(ff, d, device=dev, generator=g) * 0.05
    b1 = torch.randn(ff, device=dev, generator=g) * 0.1
    seed = torch.tensor([42], dtype=torch.int64, device=dev)
    a16 = torch.empty(M, ff, device=dev, dtype=torch.bfloat16)
    h = torch.empty(M, ff, device=dev)
    K.linear(x, W1, b1, a16, epi=L.EPI_SILU | L.EPI_STORE_PRE, Cpre=h, dropout_p=0.1, seed=seed, rng_stream=9)
    xd, wd = _deq(*_mx(x)), _deq(*_mx(W1))
    _check(h, xd @ wd.t() + b1.double(), xd.abs() @ wd.abs().t() + b1.double().abs(), 2e-5)
    monkeypatch.setattr(K._State, "fp8", False)
    K._BIG = False
    try:
        a_gen = torch.empty(M, ff, device=dev)
        K.linear(x, W1, b1, a_gen, epi=L.EPI_SILU, dropout_p=0.1, seed=seed, rng_stream=9)
    finally:
        K._BIG = True
    assert torch.equal(a_gen != 0, a16 != 0), "dropout mask differs from the generic route's"
    silu = h.double() * torch.sigmoid(h.double())
    ref_a = torch.where(a_gen != 0, silu / 0.9, torch.zeros_like(silu))
    assert torch.allclose(a16.double(), ref_a.bfloat16().double(), rtol=1e-2, atol=1e-3)
