"""Parity of the whole ver5 step (HIP path, f32 MFMA parity mode) against the CPU oracle.

The oracle (oracle/ver5.py) is pinned to the reference's own KD-head classes by golden vectors and
to NeMo's invariants; here the product (kdfm.engine.Ver5Engine, all libkdfm kernels) runs the same
seeded weights and inputs and must match losses, the mel frontend, every hooked layer output and
every trainable gradient.  Tolerances (fp32 kernels vs the oracle evaluated in float64): losses rtol 2e-4; activations
max|diff| <= 2e-3 * max|ref| + 1e-6 per tensor; gradients the same, or within 4x the float32
oracle's own distance to float64 (the step's f32 rounding noise) where that noise is larger.  The engine
runs with deterministic reductions (PARITY.deterministic: no split-K / cross-block atomics, weight
gradients in line), and once at the benchmark shape with the benchmark's schedule instead
(deterministic=False: weight gradients on the overlapped side stream, unordered reductions).
"""
import os

import pytest
import torch

from oracle import ver5 as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

# gradients that vanish analytically: a key bias shifts every score of a query row by the same
# constant (softmax-invariant); the depthwise-conv bias is removed by batch-statistics BatchNorm.
ANALYTIC_ZERO = ("self_attn.linear_k.bias", "conv.depthwise_conv.bias")


def _build(n_layers, B, N, lens, U, tl, seed=0, sub=None):
    from kdfm.config import PARITY
    from dataclasses import replace
    from kdfm.engine import Ver5Engine
    cfg = replace(PARITY, n_layers=n_layers, **(sub or {}))
    eng = Ver5Engine(cfg, "cuda", teacher_seed=seed, student_seed=seed + 1, heads_seed=seed + 2)
    g = torch.Generator().manual_seed(seed + 10)
    for name, _ in eng.bn.specs:   # non-trivial running stats for the eval-mode teacher
        if name.startswith("teacher."):
            v = (1.0 + 0.3 * torch.rand(eng.bn.P[name].shape, generator=g)) if name.endswith("running_var") else \
                0.2 * torch.randn(eng.bn.P[name].shape, generator=g)
            eng.bn.P[name].copy_(v)
    wav = 0.1 * torch.randn(B, N, generator=g)
    wl = torch.tensor(lens, dtype=torch.int64)
    tg = torch.randint(0, cfg.vocab, (B, U), generator=g)
    tgl = torch.tensor(tl, dtype=torch.int64)
    return cfg, eng, wav, wl, tg, tgl, g


def _oracle_params(cfg, eng):
    ocfg = O.StepConfig(n_layers=cfg.n_layers, subsampling=cfg.subsampling, subsampling_factor=cfg.subsampling_factor,
                        subsampling_conv_channels=cfg.subsampling_conv_channels,
                        causal_downsampling=cfg.causal_downsampling, version=cfg.version,
                        kd_loss_type=cfg.kd_loss_type, use_diffkd=cfg.use_diffkd, diffkd_steps=cfg.diffkd_steps,
                        vocab=cfg.vocab, d_teacher=cfg.d_teacher, heads_teacher=cfg.heads_teacher,
                        d_student=cfg.d_student, heads_student=cfg.heads_student, conv_kernel=cfg.conv_kernel,
                        kd_model=cfg.kd_model, xscaling=cfg.xscaling)
    p = {}
    p.update(O.frontend_buffers(ocfg))
    p.update(O.frontend_buffers(ocfg, "teacher.preprocessor.featurizer."))
    p.update(eng.student.state_dict())
    p.update(eng.teacher.state_dict())
    p.update(eng.fixed.state_dict())
    for name, _ in eng.bn.specs:
        p[name] = eng.bn.P[name].detach().cpu().clone()
    return ocfg, p


def _close(a, b, tol, what, atol=1e-6, failures=None):
    """max|a-b| <= tol*max|b| + atol.  The absolute floor covers gradients that are analytically
    zero (e.g. linear_k.bias: a per-row constant shift of the scores cancels in the softmax).
    With `failures` (a list) mismatches are collected instead of raised."""
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = b.abs().max().item()
    err = (a - b).abs().max().item()
    msg = f"{what}: max|diff| {err:.3e} vs max|ref| {scale:.3e}"
    if failures is not None:
        if not err <= tol * scale + atol:
            failures.append(msg)
        return
    assert err <= tol * scale + atol, msg


def first_conv_ok(k, mine, ref, tol=2e-3, max_rows=2, row_tol=5e-3, rel_row_tol=5e-2):
    """The subsampling's first conv (the log-mel's only consumer): its weight / bias gradient rows are
    per output channel, and a conv0 output whose pre-activation cancels to within the f32 log-mel's
    rounding (GPU FFT vs the oracle's) can take the other side of the ReLU, moving that one channel's
    row by one position's gradient (measured: 1 of 88 channels, 2.3e-3 / 3.5e-3 of max (overlapped), that
    row's own max 0.37 / 0.24 of the tensor's, every other channel within 1e-5 -- profiles/r04/conv0_diag.log).
    Accept when at most `max_rows` channels exceed `tol`, and each of them is still BOUNDED: its max error
    within `row_tol` x the tensor's max (2.5x the regular tolerance; one position's gradient is a small
    fraction of a row summed over ~10^4 positions) and, for weight rows, within `rel_row_tol` x that row's
    own max (a 10 % corruption of any one channel fails: tests/test_first_conv_bound.py)."""
    if "pre_encode.conv.0." not in k:
        return False
    m = mine.detach().double().cpu().reshape(mine.shape[0], -1)
    r = ref.detach().double().cpu().reshape(ref.shape[0], -1)
    scale = r.abs().max().item()
    err = (m - r).abs().max(1).values
    bad = err > tol * scale + 1e-6
    if bad.sum().item() > max_rows:
        return False
    if (err[bad] > row_tol * scale + 1e-6).any():
        return False
    if r.shape[1] > 1:
        row_scale = r.abs().max(1).values
        if (err[bad] > rel_row_tol * row_scale[bad] + 1e-6).any():
            return False
    return True


DW4 = dict(subsampling="dw_striding", subsampling_factor=4)
DW8C = dict(subsampling="dw_striding", subsampling_factor=8, subsampling_conv_channels=32, causal_downsampling=True)
# FastConformer layer shapes (configs[4]; fast-conformer_ctc_bpe.yaml:113-145): d_model 512, 8 heads (head dim 64),
# dw_striding x8 with 256 channels, depthwise conv kernel 9 -- student and teacher at that width
FC = dict(d_student=512, heads_student=8, d_teacher=512, heads_teacher=8, subsampling="dw_striding",
          subsampling_factor=8, subsampling_conv_channels=256, conv_kernel=9, sched_d_model=512)
# Conformer-CTC-large layer shapes (configs[3]'s student; NeMo conformer_ctc_bpe.yaml large: d_model 512,
# 8 heads, 'striding' x4 with d_model conv channels, depthwise kernel 31) -- the 512-channel striding
# subsampling runs the im2col + GEMM path (the one-kernel / implicit-GEMM kernels cover C <= 192)
CL = dict(d_student=512, heads_student=8, d_teacher=512, heads_teacher=8, sched_d_model=512)
# FastConformer-XL layer shapes (configs[4]; fast-conformer_ctc_bpe.yaml:29 XLarge row: d_model 1024, 8 heads ->
# head dim 128, conv kernel 9, xscaling False; dw_striding x8 with 256 channels, :113-125) -- student and teacher
XL = dict(d_student=1024, heads_student=8, d_teacher=1024, heads_teacher=8, subsampling="dw_striding",
          subsampling_factor=8, subsampling_conv_channels=256, conv_kernel=9, xscaling=False, sched_d_model=1024)


@pytest.mark.parametrize("n_layers,B,N,lens,U,tl,sub", [
    (2, 2, 19200, [19200, 16123], 12, [12, 7], None),
    (16, 2, 16000, [16000, 12800], 10, [10, 6], None),
    # the benchmark's utterance shape: 16.0 s (T'=401), U=100 targets, one padded utterance
    (16, 2, 256000, [256000, 200000], 100, [100, 61], None),
    # the same with the benchmark's schedule: weight gradients on the overlapped side stream and
    # unordered reductions (deterministic=False; VERDICT r2: the benchmarked schedule was never checked
    # against the oracle) -- same tolerances
    (16, 2, 256000, [256000, 200000], 100, [100, 61], dict(deterministic=False)),
    # depthwise-separable subsampling (teacher and student): x4 symmetric, x8 causal 32 channels
    (2, 2, 19200, [19200, 16123], 12, [12, 7], DW4),
    (2, 2, 19200, [19200, 16123], 8, [8, 5], DW8C),
    # other model versions through the fused engine (fm_latent_2: 6, 7; kd_crit L1: 8)
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(version=6)),
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(version=7)),
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(version=8, kd_loss_type="l1")),
    # --use_diffkd on top of ver5 (asr_train_diffm.py:326-394, 795-800)
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(use_diffkd=True)),
    # a V = 1024 BPE vocabulary (1025 decoder classes; conformer_ctc_bpe.yaml:87, SURVEY §8 V sensitivity)
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(vocab=1024)),
    # teacher as wide as the student: the two encoders (issued interleaved on two streams) must keep
    # separate workspaces (the workspace key now includes the parameter prefix)
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(d_teacher=88, heads_teacher=2)),
    # FastConformer shapes (f32 parity arithmetic)
    (2, 2, 32000, [32000, 24321], 12, [12, 7], FC),
    # Conformer-CTC-large shapes (f32 parity arithmetic)
    (2, 2, 19200, [19200, 16123], 12, [12, 7], CL),
    # FastConformer-XL shapes (f32 parity arithmetic)
    (2, 2, 32000, [32000, 24321], 12, [12, 7], XL),
    # the baseline logit-KD model family (DistilEncDecCTCModelBPE, asr_train_diffm.py:170-324): CTC + 0.1 KL
    (2, 2, 19200, [19200, 16123], 12, [12, 7], dict(kd_model="logitkd")),
], ids=["2L-1.2s", "16L-1s", "16L-16s", "16L-16s-overlapped", "2L-1.2s-dw4", "2L-1.2s-dw8-causal", "2L-1.2s-ver6", "2L-1.2s-ver7",
        "2L-1.2s-ver8-l1", "2L-1.2s-diffkd", "2L-1.2s-V1024", "2L-1.2s-equal-widths", "2L-2s-fastconformer-d512",
        "2L-1.2s-conformer-large-d512", "2L-2s-fastconformer-xl-d1024", "2L-1.2s-logitkd"])
def test_ver5_step_matches_oracle(n_layers, B, N, lens, U, tl, sub):
    from kdfm.config import sub_dims
    cfg, eng, wav, wl, tg, tgl, g = _build(n_layers, B, N, lens, U, tl, sub=sub)
    T = sub_dims(cfg, N // cfg.hop + 1)[-1][0]
    eps_rows = torch.randn(n_layers * B * T, cfg.latent, generator=g)
    ctx = eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True, eps=eps_rows.cuda())
    losses = eng.losses.detach().cpu().clone()
    sfeats = ctx["sfeats"].detach().cpu().clone()
    eng.backward(ctx)
    torch.cuda.synchronize()
    grads = eng.student.grads()

    ocfg, p32 = _oracle_params(cfg, eng)
    # The reference values come from the oracle evaluated in float64 (same restatement, higher
    # precision), so the comparison measures the kernels' f32 rounding.  The oracle is also run in
    # float32: its own distance to float64 is the f32 rounding noise of the step on a CPU, the
    # yardstick for tensors whose gradient is ill-conditioned in f32 (at 16 s the subsampling conv
    # weight gradient sums 64k cancelling terms after the 16-layer backward).
    eps_o = eps_rows.view(n_layers, B, T, cfg.latent).permute(0, 1, 3, 2)
    p = {k: (v.double() if v.is_floating_point() else v) for k, v in p32.items()}
    names = O.trainable_names(p, cfg.version, cfg.use_diffkd, cfg.kd_model)
    for k in names:
        p[k] = p[k].clone().requires_grad_(True)
        p32[k] = p32[k].clone().requires_grad_(True)
    out = O.ver5_step(p, wav.double(), wl, tg, tgl, ocfg, eps_o.double())
    out32 = O.ver5_step(p32, wav, wl, tg, tgl, ocfg, eps_o)
    g32 = dict(zip(names, torch.autograd.grad(out32["loss"], [p32[k] for k in names], allow_unused=True)))
    ref = torch.stack([out["loss"], out["ctc"], out["kl"], out["recon"], out["fm"]]).detach().float()
    torch.testing.assert_close(losses, ref, rtol=2e-4, atol=2e-4)
    for i in range(n_layers):
        _close(sfeats[i].view(B, T, -1), out["s_feats"][i], 2e-3, f"student layer {i} output")
    og = torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
    failures, report = [], []
    for k, gr in zip(names, og):
        if gr is None:
            gr = torch.zeros_like(p[k])
        if k.endswith(ANALYTIC_ZERO):
            # both sides must be rounding noise; compare against the layer's weight-grad scale
            ref_scale = grads[k.rsplit(".", 1)[0] + ".weight"].abs().max().item()
            assert grads[k].abs().max().item() <= 1e-4 * ref_scale + 1e-6, k
            assert gr.abs().max().item() <= 1e-4 * ref_scale + 1e-6, k
            continue
        mine = grads[k].detach().double().cpu()
        err = (mine - gr).abs().max().item()
        noise = ((g32[k].double() - gr).abs().max().item()) if g32.get(k) is not None else 0.0
        scale = gr.abs().max().item()
        report.append((err / max(scale, 1e-30), k, err, noise, scale))
        if not (err <= 2e-3 * scale + 1e-6 or err <= 4.0 * noise or first_conv_ok(k, mine, gr)):
            failures.append(f"grad {k}: max|diff| {err:.3e} vs max|ref| {scale:.3e} (f32 CPU noise {noise:.3e})")
    report.sort(reverse=True)
    out_dir = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out_dir):
        tag = "" if sub is None else "_" + "_".join(f"{k}{v}" for k, v in sub.items())
        with open(os.path.join(out_dir, f"step_parity_{n_layers}L_{N}{tag}.txt"), "w") as fh:
            for r in report[:25]:
                fh.write(f"{r[0]:.3e} {r[1]} err {r[2]:.3e} f32cpu-noise {r[3]:.3e} max {r[4]:.3e}\n")
    assert not failures, f"{len(failures)} gradients out of tolerance: {failures}"


def test_frontend_matches_oracle():
    from kdfm.config import PARITY
    from kdfm.frontend import FrontendConsts, frontend_forward
    from kdfm import kernels as K
    cfg = PARITY
    g = torch.Generator().manual_seed(3)
    B, N = 3, 48000
    wav = 0.2 * torch.randn(B, N, generator=g)
    wl = torch.tensor([N, 40001, 16000], dtype=torch.int64)
    fe = FrontendConsts(cfg, "cuda")
    ml = torch.empty(B, dtype=torch.int64, device="cuda")
    K.subsample_lengths(wl.cuda(), ml, None, None, cfg.hop)
    mel = frontend_forward(cfg, fe, wav.cuda(), wl.cuda(), ml, dither=0.0)
    ocfg = O.StepConfig()
    b = O.frontend_buffers(ocfg)
    ref, rl = O.preprocess(wav, wl, b["preprocessor.featurizer.window"], b["preprocessor.featurizer.fb"][0], ocfg)
    assert torch.equal(ml.cpu(), rl)
    _close(mel.cpu().transpose(1, 2), ref, 2e-4, "log-mel")


@pytest.mark.parametrize("sub", [FC, CL, XL, dict()], ids=["fastconformer-d512-h8", "conformer-large-d512-h8",
                                                           "fastconformer-xl-d1024-h8", "conformer-small"])
def test_bf16_step_matches_float64_oracle(sub):
    """The bf16 benchmark kernels (fused LN-block FFN / projections where the width has them, the fused
    rel-pos attention forward and the bwd2 backward -- at head dim 64 for the FastConformer shapes, 128 for XL --,
    bf16 weight gradients, the one-kernel striding subsampling for Conformer-small) through a whole
    2-layer step against the float64 oracle, dropout / SpecAugment / dither off, deterministic reductions.
    Tolerances are the bf16 step's (tests/test_bench_shape_gpu.py): losses rel 3e-3, layer outputs rel.
    Frobenius 1.5e-2, every gradient rel. Frobenius max(5e-2, 2.5 x the oracle's own bf16 sensitivity)."""
    _bf16_step_check(sub, 2, 32000, [32000, 24321], 12, [12, 7])


@pytest.mark.parametrize("sub,B,N,lens", [(XL, 8, 96000, [96000] * 7 + [71234]), (CL, 4, 96000, [96000, 80011, 96000, 90000])],
                         ids=["fastconformer-xl-d1024-8x6s", "conformer-large-d512-4x6s"])
def test_bf16_step_big_route_matches_float64_oracle(sub, B, N, lens, monkeypatch):
    """The same check with enough rows (>= 512) that every wide Linear of the layers -- q|k|v, out, both FFNs'
    up / down projections and the conv module's pointwise convs, their data and weight gradients -- takes the
    large-tile bf16 route (csrc/biggemm.hip) with its bf16 FFN intermediates (the work floor M N K >= 2^31 is
    lifted so the d x d products at these row counts take it too)."""
    from kdfm import kernels as K
    monkeypatch.setattr(K, "_BIG_MIN_WORK", 0.0)
    n = {"big": 0}
    orig = K.call

    def call(name, *a):
        if name == "kdfm_gemm_big":
            n["big"] += 1
        return orig(name, *a)
    monkeypatch.setattr(K, "call", call)
    _bf16_step_check(sub, B, N, lens, 12, [12, 7, 9, 5, 12, 11, 3, 8][:B], round_acts="bf16")
    assert n["big"] >= 2 * 6 * 3, n   # per layer: >= 6 wide products forward (teacher + student) + dX + dW


def test_fp8_xl_step_matches_float64_oracle(monkeypatch):
    """BASELINE.json configs[4] at its stated precision: the FastConformer-XL 2-layer step with linear_fp8 -- every
    wide Linear's forward and data gradient on MX e4m3 operands (an e8m0 scale per 32 contraction elements, block-
    scaled MFMA), the attention core and weight gradients bf16 -- against the float64 oracle.  Tolerances derived from
    the oracle's own fp8 sensitivity: the same float64 step with those products' operands
    MX-rounded (x and W; the weights everywhere else to bf16); losses rel max(3e-3, 2.5 x sens), layer outputs and
    gradients rel. Frobenius max(floor, 2.5 x sens) with the bf16 test's floors."""
    from kdfm import kernels as K
    monkeypatch.setattr(K, "_BIG_MIN_WORK", 0.0)
    n = {"fp8": 0}
    orig = K.call

    def call(name, *a):
        if name == "kdfm_gemm_big_fp8":
            n["fp8"] += 1
        return orig(name, *a)
    monkeypatch.setattr(K, "call", call)
    _bf16_step_check(dict(XL, linear_fp8=True), 8, 96000, [96000] * 7 + [71234], 12, [12, 7, 9, 5, 12, 11, 3, 8],
                     round_acts="fp8")
    assert n["fp8"] >= 2 * 6 * 2, n


class _RoundedF:
    """torch.nn.functional for the oracle with the MFMA operand rounding of the wide products: F.linear and
    pointwise (kernel 1) F.conv1d whose weight is >= 512 x 512 and whose input has >= 512 rows get their input and
    weight rounded -- to bf16, or to MX e4m3 (blocks of 32 along the contraction, block exponent
    ceil(log2(amax / 448)), kdfm_fp8_quant_mx's rule) -- straight-through for autograd.  Everything else is torch's."""

    def __init__(self, fmt):
        self.fmt = fmt
        self._F = torch.nn.functional

    def __getattr__(self, n):
        return getattr(self._F, n)

    def _q(self, t, dim=-1):
        if self.fmt == "bf16":
            q = t.bfloat16().to(t.dtype)
        else:
            q = mx_round(t.detach().movedim(dim, -1)).movedim(-1, dim).to(t.dtype)
        return t + (q - t).detach()

    def _wide(self, rows, w):
        return rows >= 512 and w.shape[0] >= 512 and w.shape[1] >= 512

    def linear(self, x, w, b=None):
        if self._wide(x.numel() // x.shape[-1], w):
            x, w = self._q(x), self._q(w)
        return self._F.linear(x, w, b)

    def conv1d(self, x, w, b=None, *a, **kw):
        if w.dim() == 3 and w.shape[-1] == 1 and x.dim() == 3 and self._wide(x.shape[0] * x.shape[2], w[:, :, 0]):
            x, w = self._q(x, 1), self._q(w, 1)   # contraction = the input channels
        return self._F.conv1d(x, w, b, *a, **kw)


def mx_round(t):
    """MX e4m3 rounding along the last dim (blocks of 32; kdfm_fp8_quant_mx): e = ceil(log2(amax / 448)) per block,
    q = e4m3(x 2^-e) 2^e, in float64."""
    shp = t.shape
    x = t.double().reshape(-1, 32)
    amax = x.abs().max(1, keepdim=True).values
    e = torch.ceil(torch.log2(amax.clamp_min(1e-300) / 448.0))
    e = torch.where(amax > 0, e, torch.full_like(e, -127.0)).clamp(-127, 127)
    sc = torch.pow(2.0, e)
    q = (x / sc).float().to(torch.float8_e4m3fn).double() * sc
    return q.reshape(shp)


def _bf16_step_check(sub, B, N, lens, U, tl, round_acts=None):
    """round_acts: also round the wide products' operands in the oracle's sensitivity run ("bf16" / "fp8", _RoundedF)
    -- the GPU rounds activations at every MFMA, not only weights."""
    n_layers = 2
    cfg, eng, wav, wl, tg, tgl, g = _build(n_layers, B, N, lens, U, tl, sub=dict(sub, math="bf16"))
    from kdfm.config import sub_dims
    T = sub_dims(cfg, N // cfg.hop + 1)[-1][0]
    eps_rows = torch.randn(n_layers * B * T, cfg.latent, generator=g)
    ctx = eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True, eps=eps_rows.cuda())
    losses = eng.losses.detach().cpu().clone()
    sfeats = ctx["sfeats"].detach().cpu().clone()
    eng.backward(ctx)
    torch.cuda.synchronize()
    grads = eng.student.grads()
    ocfg, p32 = _oracle_params(cfg, eng)
    p = {k: (v.double() if v.is_floating_point() else v) for k, v in p32.items()}
    names = O.trainable_names(p, cfg.version, cfg.use_diffkd, cfg.kd_model)
    for k in names:
        p[k] = p[k].clone().requires_grad_(True)
    eps_o = eps_rows.view(n_layers, B, T, cfg.latent).permute(0, 1, 3, 2)
    out = O.ver5_step(p, wav.double(), wl, tg, tgl, ocfg, eps_o.double())
    ref = torch.stack([out["loss"], out["ctc"], out["kl"], out["recon"], out["fm"]]).detach().double()
    rel = ((losses.double() - ref).abs() / ref.abs().clamp_min(1e-6)).max().item()
    assert round_acts or rel <= 3e-3, (rel, losses.tolist(), ref.tolist())

    def frob(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
    og = torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
    # the oracle's own sensitivity to bf16: the same float64 step with every matrix parameter rounded to
    # bf16 (the MFMA operands' rounding) -- with random weights many pre-activations sit near a ReLU /
    # softmax boundary and some gradients move by several % from that alone (cf. test_dw_striding_gpu.py)
    pb = {k: (v.detach().bfloat16().double() if (k in names and v.dim() >= 2) else v.detach()).requires_grad_(k in names)
          if v.is_floating_point() else v for k, v in p.items()}
    saved_F = O.F
    if round_acts:
        O.F = _RoundedF(round_acts)
    try:
        out_b = O.ver5_step(pb, wav.double(), wl, tg, tgl, ocfg, eps_o.double())
    finally:
        O.F = saved_F
    if round_acts:
        ref_b = torch.stack([out_b["loss"], out_b["ctc"], out_b["kl"], out_b["recon"], out_b["fm"]]).detach().double()
        sens_l = ((ref_b - ref).abs() / ref.abs().clamp_min(1e-6)).max().item()
        print(f"step losses: rel err {rel:.3e}, sensitivity {sens_l:.3e}")
        assert rel <= max(3e-3, 2.5 * sens_l), (rel, sens_l)
    # layer outputs: max(1.5e-2, 2.5 x the same sensitivity) -- at d_model 1024 (XL) the bf16-rounded weights alone
    # move the second layer's output ~0.7 %
    for i in range(n_layers):
        e = frob(sfeats[i].view(B, T, -1), out["s_feats"][i])
        sens = frob(out_b["s_feats"][i], out["s_feats"][i])
        print(f"layer {i} output: rel err {e:.3e}, sensitivity {sens:.3e}")
        assert e <= max(1.5e-2, 2.5 * sens), (i, e, sens)
    gb = torch.autograd.grad(out_b["loss"], [pb[k] for k in names], allow_unused=True)
    bad = []
    for k, gr, grb in zip(names, og, gb):
        if gr is None or k.endswith(ANALYTIC_ZERO) or gr.abs().max().item() == 0.0:
            continue
        e = frob(grads[k], gr)
        sens = frob(grb, gr) if grb is not None else 0.0
        if round_acts:
            print(f"grad {k}: rel err {e:.3e}, sensitivity {sens:.3e}")
        if e > max(5e-2, 2.5 * sens):
            bad.append((k, e, sens))
    assert not bad, bad
