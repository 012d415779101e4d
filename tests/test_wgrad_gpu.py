"""The row-parallel weight-gradient kernel (csrc/wgrad.hip, kdfm_gemm route "wgrad_rows") against
torch fp32 on the same device: every wave-tile instance, the implicit ones column (bias gradient),
alpha, accumulation into a non-zero gradient, rows that are not a multiple of the 32-row step,
multi-slice wide outputs, and the Conv1d(k=3) CONV mode with utterance boundaries.  bf16 operands,
f32 accumulation: max|diff| <= 2e-2 * max|ref|.  Also: bitwise reproducible in deterministic mode (ordered
fold), and the non-deterministic per-XCD slot accumulation equal to it up to f32 summation order."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # rows, M (dY cols), N (X cols), bias
    (12832, 88, 352, True), (12832, 352, 88, True), (12832, 264, 88, True), (12832, 176, 88, True),
    (12832, 88, 88, True), (12832, 88, 1760, False), (25600, 88, 792, True), (205312 // 8, 96, 96, True),
    (205312 // 8, 96, 176, True), (205312 // 8, 176, 96, True), (4097, 96, 88, True), (2049, 128, 20, True),
    # the decoder's 129 classes: rows of dY 4-byte aligned only, M % 4 != 0 (scalar A staging, WrGeo::ascal)
    (12832, 129, 88, True), (5003, 131, 40, False),
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
    # deterministic mode (ordered fold): a second identical call adds bitwise the same increment
    dW2 = dW0.clone()
    with K.mode("bf16", True):
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


@pytest.mark.parametrize("R,M,N", [(12832, 352, 88), (12832, 88, 352), (12832, 176, 88), (4097, 96, 88)])
def test_m_slices_bitwise(R, M, N, monkeypatch):
    """Output-row slicing (blockIdx.z, for short reductions) changes which workgroup owns an output
    row, not the row order of any sum: the sliced result equals the unsliced one bit for bit."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(7 * R + M)
    dy = torch.randn(R, M, device="cuda", generator=g)
    x = torch.randn(R, N, device="cuda", generator=g)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("KDFM_WGR_MSL", flag)
        dW, db = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
        with K.mode("bf16"):
            K.linear_dw(dy, x, dW, alpha=1.0, db=db)
        assert _route() == "wgrad_rows"
        out.append((dW, db))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


BF16_SHAPES = [  # rows, M, N, bias: multiples of 8 (8-column staging units) and of 4 only (4-column units)
    (12832, 352, 88, True), (12832, 88, 352, True), (12832, 88, 88, True), (205312 // 4, 96, 96, True),
    (4097, 264, 88, False), (12832, 84, 92, True), (3001, 20, 36, True),
]


def _bf16_ref(dy, x, alpha):
    return alpha * (dy.double().T @ x.double()), alpha * dy.double().sum(0)


@pytest.mark.parametrize("R,M,N,bias", BF16_SHAPES)
def test_wgrad_bf16_units(R, M, N, bias, monkeypatch):
    """kdfm_wgrad_bf16 (bf16 row operands): against float64 on the same bf16 values (exact products,
    f32 accumulation: 1e-5 relative), and the 8-column staging units bitwise equal to the 4-column
    ones (same LDS image, same MFMA order)."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(R * 3 + M + N)
    dy = torch.randn(R, M, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(R, N, device="cuda", generator=g).to(torch.bfloat16)
    rw, rb = _bf16_ref(dy, x, 0.75)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("KDFM_WGR_BIN8", flag)
        dW = torch.zeros(M, N, device="cuda")
        db = torch.zeros(M, device="cuda") if bias else None
        K.wgrad_bf16(dy, x, dW, db=db, alpha=0.75)
        torch.cuda.synchronize()
        assert (dW.double() - rw).abs().max().item() <= 1e-5 * rw.abs().max().item() + 1e-6
        if bias:
            assert (db.double() - rb).abs().max().item() <= 1e-5 * rb.abs().max().item() + 1e-6
        out.append((dW, db))
    assert torch.equal(out[0][0], out[1][0])
    if bias:
        assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("B,T,C", [(64, 401, 96), (9, 123, 44)])
def test_wgrad_bf16_conv_units(B, T, C, monkeypatch):
    """kdfm_wgrad_bf16_conv (SimpleDenoiser Conv1d(k=3) over utterances of T frames), 8- and
    4-column staging units, against float64 conv1d autograd on the same bf16 values."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(B * T + C)
    x = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(B, T, C, device="cuda", generator=g).to(torch.bfloat16)
    xr = x.double().transpose(1, 2).requires_grad_(True)
    W = torch.zeros(C, C, 3, dtype=torch.float64, device="cuda", requires_grad=True)
    bb = torch.zeros(C, dtype=torch.float64, device="cuda", requires_grad=True)
    out = torch.nn.functional.conv1d(xr, W, bb, padding=1)
    gW, gb = torch.autograd.grad(out, [W, bb], dy.double().transpose(1, 2))
    ref = gW.permute(0, 2, 1).reshape(C, 3 * C)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("KDFM_WGR_BIN8", flag)
        G = torch.zeros(C, 3 * C, device="cuda")
        db = torch.zeros(C, device="cuda")
        K.wgrad_bf16_conv(dy.view(B * T, C), x.view(B * T, C), G, T, db=db)
        torch.cuda.synchronize()
        assert (G.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-6
        assert (db.double() - gb).abs().max().item() <= 1e-5 * gb.abs().max().item() + 1e-6
        res.append(G)
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("nseg,seg,M,N", [(8, 205312 // 16, 96, 96), (3, 4096, 88, 352), (1, 2048, 96, 96),
                                          (16, 64, 20, 36)])
def test_wgrad_bf16_segments(nseg, seg, M, N):
    """kdfm_wgrad_bf16_seg (one launch over stacked segments, per-segment bias columns) against float64
    on the same bf16 values: dW over all rows, db[j] over segment j only."""
    from kdfm import kernels as K
    R = nseg * seg
    g = torch.Generator(device="cuda").manual_seed(nseg * 1000 + seg + M)
    dy = torch.randn(R, M, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(R, N, device="cuda", generator=g).to(torch.bfloat16)
    W0 = torch.randn(M, N + 5, device="cuda", generator=g)
    dW = W0.clone()
    db = torch.ones(nseg, M, device="cuda")
    assert K.wgrad_bf16_seg_ok(R, M, N, seg)
    K.wgrad_bf16_seg(dy, x, dW[:, :N], db, seg, alpha=-0.5)
    torch.cuda.synchronize()
    rw = -0.5 * (dy.double().T @ x.double())
    rb = 1.0 - 0.5 * dy.double().view(nseg, seg, M).sum(1)
    assert (dW[:, :N].double() - W0[:, :N].double() - rw).abs().max().item() <= 1e-5 * rw.abs().max().item() + 1e-5
    assert torch.equal(dW[:, N:], W0[:, N:])   # ldc > N: columns past N untouched
    assert (db.double() - rb).abs().max().item() <= 1e-5 * rb.abs().max().item() + 1e-5
    assert not K.wgrad_bf16_seg_ok(R + 32, M, N, seg)   # rows must be whole segments
    # the shape query agrees with the launch's preconditions even with one segment:
    # seg_rows % 32 != 0 is refused by both
    assert not K.wgrad_bf16_seg_ok(seg + 8, M, N, seg + 8)
    assert not K.wgrad_bf16_seg_ok(17 * 64, M, N, 64)    # at most 16 segments


@pytest.mark.parametrize("R,M,N,bias", [(12832, 352, 88, True), (12832, 88, 352, True), (12832, 88, 88, True),
                                        (12832, 88, 1760, False), (4097, 264, 88, False)])
def test_xcd_slots_match_ordered_fold(R, M, N, bias, monkeypatch):
    """Non-deterministic mode adds each split's tile into one of 8 per-XCD slots with float atomics
    (csrc/wgrad.hip GemmP::xslots) instead of one raw partial per split: same products, only the f32
    summation order differs -- against the deterministic ordered fold <= 1e-5 relative, for the f32
    (kdfm_gemm) and the bf16-operand (kdfm_wgrad_bf16) entry points; KDFM_WGR_XCD=0 restores the per-split
    partials bitwise."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(R + 5 * M + N)
    dy = torch.randn(R, M, device="cuda", generator=g)
    x = torch.randn(R, N, device="cuda", generator=g)
    res = {}
    for det, xcd in ((True, "0"), (False, "1"), (False, "0")):
        monkeypatch.setenv("KDFM_WGR_XCD", xcd)
        dW, db = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
        dWh, dbh = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
        with K.mode("bf16", det):
            K.linear_dw(dy, x, dW, alpha=0.5, db=db if bias else None)
            assert _route() == "wgrad_rows"
            K.wgrad_bf16(dy.to(torch.bfloat16), x.to(torch.bfloat16), dWh, db=dbh if bias else None, alpha=0.5)
        torch.cuda.synchronize()
        res[(det, xcd)] = (dW, db, dWh, dbh)
    ref = res[(True, "0")]
    for a, b in zip(res[(False, "1")], ref):
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item() + 1e-6
    for a, b in zip(res[(False, "0")], ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("R,M,N,bias", [(12832, 352, 88, True), (12832, 88, 352, True), (12832, 88, 88, True),
                                        (4097, 264, 88, False), (205312 // 2, 96, 96, True)])
def test_wgrad_bf16_pair_bitwise(R, M, N, bias):
    """kdfm_wgrad_bf16_pair: two same-shape products in one launch (2S workgroups, one fold over both)
    equal their single launches bit for bit, into row-strided outputs sharing ldc; the long-reduction
    shape (>= 64 Ki rows) takes the LDS-DMA kernel as two launches -- also bitwise."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(R + M * 3 + N)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731
    dy1, x1, dy2, x2 = mk(R, M), mk(R, N), mk(R, M), mk(R, N)
    base = torch.randn(2, M, N + 3, device="cuda", generator=g)
    bb = torch.randn(2, M, device="cuda", generator=g)
    single = base.clone()
    sb = bb.clone()
    K.wgrad_bf16(dy1, x1, single[0, :, :N], db=sb[0] if bias else None, alpha=0.5)
    K.wgrad_bf16(dy2, x2, single[1, :, :N], db=sb[1] if bias else None, alpha=0.5)
    pair = base.clone()
    pb = bb.clone()
    K.wgrad_bf16_pair(dy1, x1, pair[0, :, :N], pb[0] if bias else None, dy2, x2, pair[1, :, :N],
                      pb[1] if bias else None, alpha=0.5)
    torch.cuda.synchronize()
    assert torch.equal(single, pair)
    assert torch.equal(sb, pb)


def test_deferred_folds_bitwise():
    """kdfm_wgrad_set_fold_arena / kdfm_wgrad_fold_flush: a Conformer layer's worth of products (singles, a pair,
    a segmented product, the LDS-DMA route, a conv-mode product) with their folds queued and run in one batched
    launch equal the immediate folds bit for bit; gradients are untouched until the flush; a product whose
    partials overflow the arena folds at once; more than 24 queued products take several launches."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(11)
    mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731
    R = 12832
    prods = [(mk(R, 352), mk(R, 88), True), (mk(R, 88), mk(R, 352), True), (mk(R, 264), mk(R, 88), True),
             (mk(R, 88), mk(R, 88), False)]
    pa = (mk(R, 88), mk(R, 88), mk(R, 88), mk(R, 88))
    seg = (mk(4 * 2048, 96), mk(4 * 2048, 96))
    dma = (mk(205312, 96), mk(205312, 96))
    conv = (mk(9 * 401, 96), mk(9 * 401, 96))

    def run(outs):
        i = 0
        for dy, x, bias in prods:
            K.wgrad_bf16(dy, x, outs[i][0], db=outs[i][1] if bias else None, alpha=0.5)
            i += 1
        K.wgrad_bf16_pair(pa[0], pa[1], outs[i][0], outs[i][1], pa[2], pa[3], outs[i + 1][0], outs[i + 1][1])
        i += 2
        K.wgrad_bf16_seg(seg[0], seg[1], outs[i][0], outs[i][1], 2048)
        i += 1
        K.wgrad_bf16(dma[0], dma[1], outs[i][0], db=outs[i][1])
        i += 1
        K.wgrad_bf16_conv(conv[0], conv[1], outs[i][0], 401, db=outs[i][1])

    def fresh():
        gg = torch.Generator(device="cuda").manual_seed(5)
        shapes = [(352, 88), (88, 352), (264, 88), (88, 88), (88, 88), (88, 88), (96, 96), (96, 96), (96, 288)]
        outs = [(torch.randn(m, n, device="cuda", generator=gg), torch.randn(m, device="cuda", generator=gg))
                for m, n in shapes]
        outs[6] = (outs[6][0], torch.randn(4, 96, device="cuda", generator=gg))   # seg: one bias row per segment
        return outs

    ref = fresh()
    run(ref)
    got = fresh()
    before = [(a.clone(), b.clone()) for a, b in got]
    arena = torch.empty(40 << 20, device="cuda")
    K.wgrad_set_fold_arena(arena)
    run(got)
    assert K.wgrad_fold_pending() == 9
    torch.cuda.synchronize()
    for (a, b), (a0, b0) in zip(got, before):   # nothing folded yet
        assert torch.equal(a, a0) and torch.equal(b, b0)
    K.wgrad_fold_flush()
    assert K.wgrad_fold_pending() == 0
    torch.cuda.synchronize()
    for (a, b), (ra, rb) in zip(got, ref):
        assert torch.equal(a, ra) and torch.equal(b, rb)
    # more than one batch launch, and an arena too small for one product: that one folds at once
    got2 = [fresh() for _ in range(3)]
    for o in got2:
        run(o)
    K.wgrad_fold_flush()
    K.wgrad_set_fold_arena(None)
    small = torch.empty(1 << 20, device="cuda")
    K.wgrad_set_fold_arena(small)
    got3 = fresh()
    run(got3)
    assert 0 < K.wgrad_fold_pending() < 9
    K.wgrad_fold_flush()
    K.wgrad_set_fold_arena(None)
    torch.cuda.synchronize()
    for o in got2 + [got3]:
        for (a, b), (ra, rb) in zip(o, ref):
            assert torch.equal(a, ra) and torch.equal(b, rb)
    # two queued products adding into the same gradient (the heads' layer halves) fold in queue order
    dWi = torch.randn(88, 88, device="cuda", generator=g)
    dbi = torch.randn(88, device="cuda", generator=g)
    dWd, dbd = dWi.clone(), dbi.clone()
    for k in range(3):
        K.wgrad_bf16(prods[3][0], pa[k], dWi, db=dbi, alpha=0.25 * (k + 1))
    K.wgrad_set_fold_arena(arena)
    for k in range(3):
        K.wgrad_bf16(prods[3][0], pa[k], dWd, db=dbd, alpha=0.25 * (k + 1))
    K.wgrad_fold_flush()
    K.wgrad_set_fold_arena(None)
    torch.cuda.synchronize()
    assert torch.equal(dWi, dWd) and torch.equal(dbi, dbd)


@pytest.mark.parametrize("R,M,N", [(12832, 88, 1760), (25600, 88, 792), (12831, 96, 800)])
def test_xcd_grouped_slices_bitwise(R, M, N, monkeypatch):
    """The XCD-grouped dispatch order of multi-slice products (WrGeo::xgrp: a split's column slices on one
    XCD) renumbers the grid, nothing else: bitwise the plain order's result, single and paired launches,
    and the 3x3 stride-2 gather (conv2's weight gradient, 3 column slices)."""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(R + 5 * N)
    dy = torch.randn(R, M, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(R, N, device="cuda", generator=g).to(torch.bfloat16)
    dy2 = torch.randn(R, M, device="cuda", generator=g).to(torch.bfloat16)
    x2 = torch.randn(R, N, device="cuda", generator=g).to(torch.bfloat16)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("KDFM_WGR_XGRP", flag)
        dW, db = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
        K.wgrad_bf16(dy, x, dW, db=db, alpha=0.5)
        dWa, dba = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
        dWb, dbb = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
        K.wgrad_bf16_pair(dy, x, dWa, dba, dy2, x2, dWb, dbb, alpha=0.5)
        out.append((dW, db, dWa, dba, dWb, dbb))
    torch.cuda.synchronize()
    rw = 0.5 * (dy.double().T @ x.double())
    assert (out[1][0].double() - rw).abs().max().item() <= 1e-5 * rw.abs().max().item() + 1e-6
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,T1,F1", [(4, 801, 80), (3, 41, 40)])
def test_xcd_grouped_s2conv_bitwise(B, T1, F1, monkeypatch):
    from kdfm import kernels as K
    C = 88
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    g = torch.Generator().manual_seed(T1 + F1)
    X = torch.randn(B * T1 * F1, C, generator=g).bfloat16().cuda()
    dY = torch.randn(B * T2 * F2, C, generator=g).bfloat16().cuda()
    lin = torch.tensor([T1 - 5 * b for b in range(B)], dtype=torch.int64).cuda()
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("KDFM_WGR_XGRP", flag)
        dW, db = torch.zeros(C, 9 * C, device="cuda"), torch.zeros(C, device="cuda")
        K.wgrad_bf16_s2conv(dY, X, lin, dW, db, B, T1, F1, C)
        out.append((dW, db))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
