"""GPU numerics of the fused striding-subsampling forward (csrc/subsample.hip): direct conv1 with
the frame masks of SURVEY.md A.3, and the implicit-GEMM conv2 (bf16 MFMA).  Reference: torch CPU
f32 conv2d of the same (masked) inputs; conv2 is compared on the bf16-rounded operands it consumes
(tolerance 2e-3 of max |ref|: f32 accumulation order only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from kdfm import kernels
    return kernels


def _bf(t):
    return t.to(torch.bfloat16).float()


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _lens(L):
    return (L - 1) // 2 + 1


@pytest.mark.parametrize("C", [88, 176, 32, 64])
def test_subsample_fused_forward(K, C):
    g = torch.Generator().manual_seed(C)
    B, Tm, Fq = 3, 57, 80
    mel = torch.randn(B, Tm, Fq, generator=g)
    mel_len = torch.tensor([Tm, 40, 23], dtype=torch.int64)
    len1 = _lens(mel_len)
    len2 = _lens(len1)
    w0 = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b0 = torch.randn(C, generator=g) * 0.1
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    b2 = torch.randn(C, generator=g) * 0.1
    T1, F1 = _lens(Tm), _lens(Fq)
    T2, F2 = _lens(T1), _lens(F1)

    # reference (CPU f32)
    x = mel.clone()
    for b in range(B):
        x[b, mel_len[b]:] = 0
    y1 = F.relu(F.conv2d(x[:, None], w0, b0, stride=2, padding=1))          # (B, C, T1, F1)
    for b in range(B):
        y1[b, :, len1[b]:] = 0
    y2 = F.relu(F.conv2d(_bf(y1), _bf(w2), b2, stride=2, padding=1))       # (B, C, T2, F2)
    for b in range(B):
        y2[b, :, len2[b]:] = 0

    dev = "cuda"
    y1b = torch.empty(B * T1 * F1, C, device=dev, dtype=torch.bfloat16)
    y1f = torch.empty(B * T1 * F1, C, device=dev)
    K.subsample_conv1(mel.to(dev), mel_len.to(dev), len1.to(dev), w0.to(dev), b0.to(dev), y1b, y1f, B, Tm, Fq, C)
    y1_ref = y1.permute(0, 2, 3, 1).reshape(B * T1 * F1, C)
    torch.testing.assert_close(y1f.cpu(), y1_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y1b.float().cpu(), _bf(y1_ref), rtol=1e-2, atol=1e-2)

    wb = torch.empty(K.subsample_wprep_elems(C), device=dev, dtype=torch.bfloat16)
    K.subsample_wprep(w2.to(dev), wb)
    out = torch.full((B * T2 * F2, C), float("nan"), device=dev)
    # feed the exact bf16 y1 of the reference so only accumulation order differs
    K.subsample_conv2(_bf(y1_ref).to(torch.bfloat16).to(dev), len2.to(dev), wb, b2.to(dev), out, B, T1, F1, C)
    ref = y2.permute(0, 2, 3, 1).reshape(B * T2 * F2, C)
    err = (out.cpu() - ref).abs().max().item()
    assert err <= 2e-3 * ref.abs().max().item() + 1e-6, err


@pytest.mark.parametrize("C,Tm,lens", [(88, 57, (57, 40, 23)), (176, 57, (57, 40, 23)), (96, 200, (200, 199, 17)),
                                        (192, 73, (73, 8, 3)), (176, 1601, (1601, 1000, 333)),
                                        (88, 1601, (1601, 1600, 5))])
def test_subsample_one_kernel_forward(K, C, Tm, lens):
    """kdfm_subsample_fused (conv1 on the fly in LDS by hi/lo-split bf16 MFMA, conv2 implicit GEMM):
    * y1 (the student's side output) against the f32 conv1 of the masked mel rounded to bf16: the f32
      values agree to ~2^-16 relative, so every bf16 y1 is the reference's or its bf16 neighbour (ties
      at a rounding boundary), >= 99 % exactly equal, masked rows / padding exactly 0;
    * y2 against float64 conv2d(stride 2, pad 1) of the kernel's own bf16 y1 with the bf16 weights,
      + bias, ReLU, len2 mask: max error <= 1e-4 of max |ref| (f32 accumulation order only);
    * the teacher form (no y1 output) gives the identical y2 bit for bit.
    Shapes: output rows not a multiple of the 8-row workgroup strip, the bench utterance (T_mel 1601),
    ragged lengths down to a 3-frame utterance."""
    g = torch.Generator().manual_seed(C + Tm)
    B, Fq = 3, 80
    mel = torch.randn(B, Tm, Fq, generator=g)
    mel_len = torch.tensor(lens, dtype=torch.int64)
    len1 = _lens(mel_len)
    len2 = _lens(len1)
    w0 = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b0 = torch.randn(C, generator=g) * 0.1
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    b2 = torch.randn(C, generator=g) * 0.1
    T1, F1 = _lens(Tm), _lens(Fq)
    T2, F2 = _lens(T1), _lens(F1)
    dev = "cuda"
    wp = torch.empty(K.subsample_fused_wprep_elems(C), device=dev, dtype=torch.bfloat16)
    K.subsample_fused_wprep(w0.cuda(), w2.cuda(), wp)
    y1 = torch.full((B * T1 * F1, C), float("nan"), device=dev).bfloat16()
    y2 = torch.full((B * T2 * F2, C), float("nan"), device=dev)
    args = (mel.cuda(), mel_len.cuda(), len1.cuda(), len2.cuda(), wp, b0.cuda(), b2.cuda())
    K.subsample_fused(*args, y2, y1, B, Tm, Fq, C)
    y2t = torch.full_like(y2, float("nan"))
    K.subsample_fused(*args, y2t, None, B, Tm, Fq, C)
    torch.cuda.synchronize()
    assert torch.equal(y2, y2t)
    # conv1 reference (f32, masked)
    x = mel.clone()
    for b in range(B):
        x[b, mel_len[b]:] = 0
    r1 = F.relu(F.conv2d(x.double()[:, None], w0.double(), b0.double(), stride=2, padding=1))
    for b in range(B):
        r1[b, :, len1[b]:] = 0
    r1 = r1.permute(0, 2, 3, 1).reshape(B * T1 * F1, C)
    # |x| * |w| conv: the hi/lo products carry ~2^-16 of it, which dominates the bf16 rounding of a y1
    # whose taps cancel to near zero
    ra = F.conv2d(x.double().abs()[:, None], w0.double().abs(), b0.double().abs(), stride=2, padding=1)
    ra = ra.permute(0, 2, 3, 1).reshape(B * T1 * F1, C)
    got1 = y1.float().cpu()
    assert torch.isfinite(got1).all()
    d = (got1.double() - r1).abs()
    assert (d <= 2.0 ** -7 * r1.abs() + 2.0 ** -14 * ra + 1e-7).all(), d.max().item()
    exact = (got1 == r1.float().bfloat16().float()).double().mean().item()
    assert exact >= 0.99, exact
    # masked rows (t1 >= len1) exactly 0; a ReLU-clipped position may come out as a tiny positive value
    # when its pre-activation cancels to within the hi/lo error (bounded above)
    masked = torch.zeros(B, T1, F1, C, dtype=torch.bool)
    for b in range(B):
        masked[b, len1[b]:] = True
    masked = masked.reshape(B * T1 * F1, C)
    assert got1[masked].abs().max().item() == 0.0 if masked.any() else True
    # conv2 reference on the kernel's own bf16 y1 and the bf16 weights
    y1d = got1.double().view(B, T1, F1, C).permute(0, 3, 1, 2)
    r2 = F.relu(F.conv2d(y1d, _bf(w2).double(), b2.double(), stride=2, padding=1))
    for b in range(B):
        r2[b, :, len2[b]:] = 0
    r2 = r2.permute(0, 2, 3, 1).reshape(B * T2 * F2, C)
    got2 = y2.cpu().double()
    assert torch.isfinite(got2).all()
    err = (got2 - r2).abs().max().item()
    assert err <= 1e-4 * r2.abs().max().item() + 1e-6, err


def test_subsample_bench_shape_matches_im2col_path(K):
    """The fused path and the im2col+GEMM path (kept for f32 parity mode) agree at the bench shape
    of one utterance (T_mel = 1601, d = 176)."""
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(0)
    B, Tm, Fq, C = 2, 1601, 80, 176
    dev = "cuda"
    mel = torch.randn(B, Tm, Fq, device=dev, generator=g)
    mel_len = torch.tensor([Tm, 1000], dtype=torch.int64, device=dev)
    len1 = (mel_len - 1) // 2 + 1
    len2 = (len1 - 1) // 2 + 1
    w0 = torch.randn(C, 9, device=dev, generator=g) * 0.3
    b0 = torch.randn(C, device=dev, generator=g) * 0.1
    w2 = torch.randn(C, C, 9, device=dev, generator=g) * 0.02
    b2 = torch.randn(C, device=dev, generator=g) * 0.1
    T1, F1 = _lens(Tm), _lens(Fq)
    T2, F2 = _lens(T1), _lens(F1)
    y1b = torch.empty(B * T1 * F1, C, device=dev, dtype=torch.bfloat16)
    y1f = torch.empty(B * T1 * F1, C, device=dev)
    K.subsample_conv1(mel, mel_len, len1, w0, b0, y1b, y1f, B, Tm, Fq, C)
    wb = torch.empty(K.subsample_wprep_elems(C), device=dev, dtype=torch.bfloat16)
    K.subsample_wprep(w2, wb)
    y2 = torch.empty(B * T2 * F2, C, device=dev)
    K.subsample_conv2(y1b, len2, wb, b2, y2, B, T1, F1, C)
    # im2col path on the same bf16 y1
    cols1 = torch.empty(B * T2 * F2, 9 * C, device=dev)
    K.im2col_3x3s2(y1b.float().contiguous(), len1, cols1, B, T1, F1, C)
    ref = torch.empty_like(y2)
    K.linear(cols1, w2.view(C, 9 * C), b2, ref, epi=_lib.EPI_RELU, rowmask=(len2, T2, F2), math="f32")
    # the f32 path sees f32 weights; the fused path bf16 weights -> bf16-level tolerance
    err = (y2 - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("C,T1,F1", [(88, 401, 40), (88, 37, 13), (16, 29, 11), (32, 30, 40), (64, 7, 5)])
def test_subsample_conv2_dgrad_direct(K, C, T1, F1):
    """kdfm_subsample_conv2_dgrad (parity-class transposed conv, bf16 MFMA) against the float64
    gradient of conv2d(stride 2, pad 1) wrt its input times ReLU'(y1), on bf16-rounded dy2 / W (the
    operands the kernel consumes; y1 is passed as the bf16 copy the engine saves, only its sign is read): rel. Frobenius <= 1e-5 (f32 accumulation only); frames where
    y1 == 0 (ReLU'd or masked) get exactly 0."""
    g = torch.Generator().manual_seed(C + T1)
    B = 2
    T2, F2 = _lens(T1), _lens(F1)
    y1 = torch.relu(torch.randn(B, T1, F1, C, generator=g))
    y1[1, T1 // 2:] = 0.0                                   # masked frames of a shorter utterance
    dy2 = torch.randn(B, T2, F2, C, generator=g)
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    x = torch.zeros(B, C, T1, F1, dtype=torch.float64, requires_grad=True)
    out = F.conv2d(x, _bf(w2).double(), stride=2, padding=1)
    (gx,) = torch.autograd.grad(out, x, _bf(dy2).double().permute(0, 3, 1, 2))
    ref = gx.permute(0, 2, 3, 1) * (y1 > 0).double()
    wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
    K.subsample_dgrad_wprep(w2.cuda(), wt)
    dy1 = torch.full((B * T1 * F1, C), float("nan"), device="cuda")
    K.subsample_conv2_dgrad(dy2.cuda().reshape(-1, C), wt, y1.cuda().reshape(-1, C).bfloat16(), dy1, B, T1, F1, C)
    torch.cuda.synchronize()
    got = dy1.cpu().double().view(B, T1, F1, C)
    assert torch.isfinite(got).all()
    err = ((got - ref).norm() / ref.norm()).item()
    assert err <= 1e-5, err
    assert got[y1 == 0].abs().max().item() == 0.0


def test_im2col_tapmajor_bf16_matches_f32_im2col(K):
    """kdfm_im2col_3x3s2_tm_bf16 = the f32 im2col (columns c*9 + tap) re-ordered to tap*C + c and
    rounded to bf16, including the len_in frame mask: bit-exact."""
    g = torch.Generator().manual_seed(7)
    B, T1, F1, C = 3, 41, 40, 88
    X = torch.randn(B * T1 * F1, C, generator=g).cuda()
    lin = torch.tensor([41, 30, 9], dtype=torch.int64).cuda()
    T2, F2 = _lens(T1), _lens(F1)
    ref = torch.empty(B * T2 * F2, 9 * C, device="cuda")
    K.im2col_3x3s2(X, lin, ref, B, T1, F1, C)
    got = torch.empty(B * T2 * F2, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.im2col_3x3s2_tm_bf16(X, lin, got, B, T1, F1, C)
    torch.cuda.synchronize()
    want = ref.view(-1, C, 9).transpose(1, 2).reshape(-1, 9 * C).bfloat16()
    assert torch.equal(got, want)


@pytest.mark.parametrize("B,T1,F1,C,masked", [(3, 41, 40, 88, True), (2, 37, 39, 88, False), (4, 9, 7, 32, True),
                                              (2, 401, 39, 88, True)])
def test_s2conv_wgrad_gather_equals_im2col(K, B, T1, F1, C, masked):
    """kdfm_wgrad_bf16_s2conv (the conv2 weight gradient gathered straight from the bf16 y1) = kdfm_wgrad_bf16
    over kdfm_im2col_3x3s2_tm_from_bf16's column matrix, bit for bit (same split plan and fold order), with
    and without the len_in frame mask, and with the folds deferred to an arena."""
    g = torch.Generator().manual_seed(11 + T1)
    T2, F2 = _lens(T1), _lens(F1)
    rows = B * T2 * F2
    X = torch.randn(B * T1 * F1, C, generator=g).bfloat16().cuda()
    dY = torch.randn(rows, C, generator=g).bfloat16().cuda()
    lin = torch.tensor([T1 - 3 * b if T1 - 3 * b > 0 else 1 for b in range(B)], dtype=torch.int64).cuda() if masked \
        else None
    cols = torch.empty(rows, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.im2col_3x3s2_tm_bf16(X, lin, cols, B, T1, F1, C)
    dW0 = torch.randn(C, 9 * C, generator=g).cuda()
    db0 = torch.randn(C, generator=g).cuda()
    dW1, db1 = dW0.clone(), db0.clone()
    K.wgrad_bf16(dY, cols, dW0, db=db0)
    K.wgrad_bf16_s2conv(dY, X, lin, dW1, db1, B, T1, F1, C)
    torch.cuda.synchronize()
    assert torch.equal(dW1, dW0) and torch.equal(db1, db0)
    dW2, db2 = dW0.clone(), db0.clone()
    arena = torch.empty(1 << 24, device="cuda")
    K.wgrad_set_fold_arena(arena)
    K.wgrad_bf16_s2conv(dY, X, lin, dW2, db2, B, T1, F1, C)
    K.wgrad_fold_flush()
    K.wgrad_set_fold_arena(None)
    dW3, db3 = dW0.clone(), db0.clone()
    K.wgrad_bf16(dY, cols, dW3, db=db3)
    torch.cuda.synchronize()
    assert torch.equal(dW2, dW3) and torch.equal(db2, db3)


@pytest.mark.parametrize("C,Tm,Fm", [(88, 801, 80), (88, 75, 27), (32, 61, 80), (64, 13, 9)])
def test_subsample_dgrad_fused_conv0_wgrad(K, C, Tm, Fm):
    """kdfm_subsample_conv2_dgrad_w0: conv0's weight / bias gradient accumulated in the conv2 data
    gradient's epilogue equals the float64 conv0 weight gradient of the same dy1 (the kernel's own
    dy1, also written) over the mel frames with frames t >= mel_len zeroed: rel. Frobenius <= 1e-5
    (f32 sums over ~1e6 positions, ordered per-workgroup fold)."""
    g = torch.Generator().manual_seed(C + Tm)
    B = 3
    T1, F1 = _lens(Tm), _lens(Fm)
    T2, F2 = _lens(T1), _lens(F1)
    mel = torch.randn(B, Tm, Fm, generator=g)
    mel_len = torch.tensor([Tm, Tm - Tm // 3, Tm // 2], dtype=torch.int64)
    y1 = torch.relu(torch.randn(B, T1, F1, C, generator=g))
    for b in range(B):   # conv1 output rows past the subsampled length are masked (zero)
        y1[b, (int(mel_len[b]) - 1) // 2 + 1:] = 0.0
    dy2 = torch.randn(B, T2, F2, C, generator=g)
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
    K.subsample_dgrad_wprep(w2.cuda(), wt)
    dy1 = torch.empty(B * T1 * F1, C, device="cuda")
    dw0 = torch.full((C, 9), 0.5, device="cuda")
    db0 = torch.zeros(C, device="cuda")
    K.subsample_conv2_dgrad_w0(dy2.cuda().reshape(-1, C), wt, y1.cuda().reshape(-1, C).bfloat16(), B, T1, F1, C,
                               mel.cuda(), mel_len.cuda(), Tm, Fm, 1, dw0, db0, dy1=dy1)
    torch.cuda.synchronize()
    d1 = dy1.cpu().double().view(B, T1, F1, C).permute(0, 3, 1, 2)
    xm = mel.double().clone()
    for b in range(B):
        xm[b, int(mel_len[b]):] = 0.0
    x = xm[:, None]
    w = torch.zeros(C, 1, 3, 3, dtype=torch.float64, requires_grad=True)
    bias = torch.zeros(C, dtype=torch.float64, requires_grad=True)
    out = F.conv2d(x, w, bias, stride=2, padding=1)
    gw, gb = torch.autograd.grad(out, [w, bias], d1)
    assert _rel(dw0.cpu() - 0.5, gw.view(C, 9)) <= 1e-5
    assert _rel(db0.cpu(), gb) <= 1e-5


@pytest.mark.parametrize("C,Tm,Fm", [(88, 801, 80), (88, 75, 27), (32, 61, 80)])
def test_subsample_dgrad_bf16_dy2_equals_f32(K, C, Tm, Fm):
    """kdfm_subsample_conv2_dgrad_w0_h (dy2 read as bf16) against kdfm_subsample_conv2_dgrad_w0 fed the same
    values in f32: the f32 kernel rounds each dy2 fragment to bf16 on load, so on bf16-exact dy2 the two run
    the same MFMAs on the same operands -- dy1, dW0 and db0 bitwise equal."""
    g = torch.Generator().manual_seed(7 * C + Tm)
    B = 3
    T1, F1 = _lens(Tm), _lens(Fm)
    T2, F2 = _lens(T1), _lens(F1)
    mel = torch.randn(B, Tm, Fm, generator=g).cuda()
    mel_len = torch.tensor([Tm, Tm - Tm // 3, Tm // 2], dtype=torch.int64).cuda()
    y1 = torch.relu(torch.randn(B * T1 * F1, C, generator=g)).cuda().bfloat16()
    dy2h = torch.randn(B * T2 * F2, C, generator=g).cuda().bfloat16()
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
    K.subsample_dgrad_wprep(w2.cuda(), wt)
    outs = []
    for h in (False, True):
        dy1 = torch.empty(B * T1 * F1, C, device="cuda")
        dw0 = torch.full((C, 9), 0.25, device="cuda")
        db0 = torch.zeros(C, device="cuda")
        if h:
            K.subsample_conv2_dgrad_w0_h(dy2h, wt, y1, B, T1, F1, C, mel, mel_len, Tm, Fm, 1, dw0, db0, dy1=dy1)
        else:
            K.subsample_conv2_dgrad_w0(dy2h.float(), wt, y1, B, T1, F1, C, mel, mel_len, Tm, Fm, 1, dw0, db0, dy1=dy1)
        outs.append((dy1, dw0, db0))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rows,d,F2,C", [(12832, 88, 20, 88), (300, 88, 20, 88), (77, 40, 5, 36), (1000, 128, 4, 64)])
def test_ss_out_dgrad_matches_linear_dx(K, rows, d, F2, C):
    """kdfm_ss_out_dgrad: the subsampling output Linear's data gradient with the ReLU' of the conv2 output, as
    bf16: against the f32 product of the bf16-rounded dlin and W (what kdfm_gemm's bf16 math multiplies) with
    the mask, rounded to bf16 -- equal but for f32 accumulation order (a bf16 rounding may flip: within one bf16
    ulp, 2^-8 relative), masked entries exactly 0."""
    g = torch.Generator().manual_seed(rows + d)
    ncols = F2 * C
    dlin = torch.randn(rows, d, generator=g)
    W = torch.randn(d, ncols, generator=g) / d ** 0.5
    y2 = torch.randn(rows, ncols, generator=g)
    wt = torch.empty(K.ss_out_wprep_elems(d, ncols), device="cuda", dtype=torch.bfloat16)
    K.ss_out_wprep(W.cuda(), wt)
    out = torch.empty(rows, ncols, device="cuda", dtype=torch.bfloat16)
    K.ss_out_dgrad(dlin.cuda(), wt, y2.cuda(), out)
    torch.cuda.synchronize()
    ref = (_bf(dlin).double() @ _bf(W).double()) * (y2 > 0).double()
    got = out.float().double().cpu()
    assert torch.equal(got[y2 <= 0], torch.zeros_like(got[y2 <= 0]))
    err = (got - ref).abs()
    assert (err <= ref.abs() * 2.0 ** -8 + 1e-6).all(), err.max().item()


@pytest.mark.parametrize("C,Tm,lens", [(88, 1601, (1601, 1600, 5)), (88, 57, (57, 40, 23)), (176, 73, (73, 8, 3))])
def test_subsample_padded_y1_rows(K, C, Tm, lens):
    """kdfm_subsample_fused with y1 rows padded to whole 32-channel chunks (ldy1 = 32 ceil(C / 32), the training
    step's layout) against the unpadded form: y2 and y1[:, :C] bitwise equal, the padding channels exactly 0;
    its consumers over the padded rows -- the conv2 weight gradient gathered from y1 (kdfm_wgrad_bf16_s2conv) and
    the conv2 data gradient with the fused conv0 weight gradient (kdfm_subsample_conv2_dgrad_w0_h, its ReLU' read
    from y1) -- bitwise equal to the same calls over the unpadded y1."""
    g = torch.Generator().manual_seed(3 * C + Tm)
    B, Fq = 3, 80
    mel = torch.randn(B, Tm, Fq, generator=g).cuda()
    mel_len = torch.tensor(lens, dtype=torch.int64).cuda()
    len1 = _lens(mel_len)
    len2 = _lens(len1)
    w0 = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b0 = (torch.randn(C, generator=g) * 0.1).cuda()
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    b2 = (torch.randn(C, generator=g) * 0.1).cuda()
    T1, F1 = _lens(Tm), _lens(Fq)
    T2, F2 = _lens(T1), _lens(F1)
    ld = -(-C // 32) * 32
    wp = torch.empty(K.subsample_fused_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
    K.subsample_fused_wprep(w0.cuda(), w2.cuda(), wp)
    args = (mel, mel_len, len1, len2, wp, b0, b2)
    y1u = torch.full((B * T1 * F1, C), float("nan"), device="cuda").bfloat16()
    y2u = torch.full((B * T2 * F2, C), float("nan"), device="cuda")
    K.subsample_fused(*args, y2u, y1u, B, Tm, Fq, C)
    y1p = torch.full((B * T1 * F1, ld), float("nan"), device="cuda").bfloat16()
    y2p = torch.full((B * T2 * F2, C), float("nan"), device="cuda")
    K.subsample_fused(*args, y2p, y1p, B, Tm, Fq, C)
    torch.cuda.synchronize()
    assert torch.equal(y2p, y2u)
    assert torch.equal(y1p[:, :C], y1u)
    if ld > C:
        assert torch.equal(y1p[:, C:].float(), torch.zeros(B * T1 * F1, ld - C, device="cuda"))
    if C > 96:   # the consumers run for the trained student's widths
        return
    dY = torch.randn(B * T2 * F2, C, generator=g).bfloat16().cuda()
    outs = []
    for y1 in (y1u, y1p):
        dW = torch.zeros(C, 9 * C, device="cuda")
        db = torch.zeros(C, device="cuda")
        K.wgrad_bf16_s2conv(dY, y1, len1, dW, db, B, T1, F1, C)
        outs.append((dW, db))
    if K.subsample_dgrad_supported(C):
        wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
        K.subsample_dgrad_wprep(w2.cuda(), wt)
        for i, y1 in enumerate((y1u, y1p)):
            dy1 = torch.empty(B * T1 * F1, C, device="cuda")
            dw0 = torch.zeros(C, 9, device="cuda")
            db0 = torch.zeros(C, device="cuda")
            K.subsample_conv2_dgrad_w0_h(dY, wt, y1, B, T1, F1, C, mel, mel_len, Tm, Fq, 1, dw0, db0, dy1=dy1)
            outs[i] = outs[i] + (dy1, dw0, db0)
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
