"""Conformer encoder forward/backward on libkdfm kernels.

Reference path: NeMo ConformerEncoder.forward_internal (conformer_encoder.py:595-761) with
ConvSubsampling 'striding' (built :381-390, called :635), RelPositionalEncoding (:422-429, :658),
_create_masks (:796-850) and 16 ConformerLayers (:450-472, :677-692) whose sources are absent from
the snapshot (SURVEY.md Appendix A.3-A.8 restates them):
  r = x + 0.5*drop(FF1(LN1 x)); r += drop(MHSA(LN2 r)); r += drop(Conv(LN3 r)); r += 0.5*drop(FF2(LN4 r));
  out = LN5(r)
Layout: channels-last rows = (utterance, frame); every per-layer output is written straight into
slot i of a (n_layers, B*T', d) buffer — the tensors the reference's forward hooks capture
(asr_train_diffm.py:584-596) — so the KD heads consume all layers as one row batch.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib
from . import kernels as K
from .overlap import WGRAD
from .config import Ver5Config, sub_channels, sub_dims, sub_pad, sub_stages

# dropout site ids (rng stream = model_salt * 4096 + layer * 16 + site)
SITE_FF1_ACT, SITE_FF1_OUT, SITE_ATT_P, SITE_ATT_OUT, SITE_CONV_OUT, SITE_FF2_ACT, SITE_FF2_OUT = range(7)
SITE_PRE = 15


# bf16 math: attention backward through the fused kernels of csrc/attn_bwd.hip (KDFM_ATTN_BWD_FUSED=0:
# the unfused dPd / dAC / dBD path; the f32 parity mode always takes it)
_ATTN_BWD_FUSED = __import__("os").environ.get("KDFM_ATTN_BWD_FUSED", "1") == "1"
# ...in the bwd2 form (default): the forward saves only the per-row log-sum-exp, the dQ kernel writes the bf16
# score gradient dS and dropped-out probabilities Pd, and dK / dV / dPpos are plain products over them
# (KDFM_ATTN_BWD2=0: the forward saves bf16 p~ and block maxima, dK / dV / dPpos recompute dS from them)
_ATTN_BWD2 = __import__("os").environ.get("KDFM_ATTN_BWD2", "1") == "1"
# bf16 math: the layer backward's same-shape weight gradients (feed_forward2 / feed_forward1 linear2 and
# linear1, pointwise_conv2 with linear_out) leave as paired launches (kdfm_wgrad_bf16_pair, each product
# bitwise its single launch's); KDFM_WGRAD_PAIRS=0: one launch per product
_WGRAD_PAIRS = __import__("os").environ.get("KDFM_WGRAD_PAIRS", "1") == "1"
# bf16 math, single-pass forward (bwd2 training / inference): the attention forward over prepared bf16 operands
# (csrc/attn_fwd3.hip: keys / values centred and tiled once per layer, the positional band once per encoder, LDS-DMA
# staging, rel_shift by lane permutes) -- bitwise the register-staged kernel's O / lse (KDFM_ATTN_FWD3=0: that kernel)
_ATTN_FWD3 = __import__("os").environ.get("KDFM_ATTN_FWD3", "1") == "1"
# ... and the bwd2 dQ kernel over the same prepared operands, kept from the forward (KDFM_ATTN_DQ3=0: it stages
# K / V / the band from qkv / pos itself)
_ATTN_DQ3 = __import__("os").environ.get("KDFM_ATTN_DQ3", "1") == "1"
# bf16 math: the encoder backward defers its layers' weight-gradient folds and folds each layer's products in one
# launch (kdfm_wgrad_set_fold_arena / kdfm_wgrad_fold_flush; bitwise the per-product folds).  KDFM_FOLD_DEFER=0:
# a fold launch per product (pair)
_FOLD_DEFER = __import__("os").environ.get("KDFM_FOLD_DEFER", "1") == "1"
_FOLD_ARENA_FLOATS = 64 << 20   # 256 MB: a layer's per-split partials at the bench shape are ~18M floats, the heads' ~40M
# (larger shapes -- the XL layers -- grow it: encoder_backward reads the library's demand / fallback counters before
# it ends deferral and fold_arena sizes the next step's arena from them)


def _attn_fused_ok(dk, save):
    """bf16 math: the fused rel-pos attention (csrc/attn_fused.hip, attn_bwd.hip).  Head dims <= 64 in every
    backward form; up to 128 (FastConformer-XL: d_model 1024 / 8 heads) with the bwd2 backward, whose forward
    keeps only the per-row log-sum-exp."""
    if K.get_math() != "bf16":
        return False
    if dk <= 64:
        return True
    return dk <= 128 and (not save or (_ATTN_BWD_FUSED and _ATTN_BWD2))


def _stream(salt, layer, site):
    return salt * 4096 + (layer + 1) * 16 + site


class EncoderShapes:
    def __init__(self, cfg: Ver5Config, B: int, T_mel: int, d: int, h: int):
        self.B, self.Tm, self.d, self.h = B, T_mel, d, h
        self.dk = d // h
        self.C = sub_channels(cfg, d)
        self.stages = sub_dims(cfg, T_mel)      # [(T, F)] of the subsampling input and stage outputs
        self.pad = sub_pad(cfg)[0]
        self.T1, self.F1 = self.stages[1]
        self.T, self.F2 = self.stages[-1]       # F2: features per frame at the subsampling output
        self.rows = B * self.T
        self.ff = cfg.ff_expansion * d


def compute_lengths(cfg: Ver5Config, wav_len, mel_len, len1, len2, hop):
    """Frame lengths of one batch: mel_len = L // hop, then the subsampling stages.  'striding':
    len1 / len2 = after stage 1 / 2 (one kernel).  'dw_striding': len1 = (stages, B) lengths of every
    stage output and len2 = its last row (a view), both returned."""
    if cfg.subsampling == "striding":
        K.subsample_lengths(wav_len, mel_len, len1, len2, hop)
        return len1, len2
    K.subsample_lengths(wav_len, mel_len, None, None, hop)
    n = sub_stages(cfg)
    lens = torch.empty(n, mel_len.numel(), dtype=torch.int64, device=mel_len.device)
    pl, pr = sub_pad(cfg)
    prev = mel_len
    for s in range(n):
        K.conv_lengths(prev, lens[s], pl + pr, 3, 2)
        prev = lens[s]
    return lens, lens[n - 1]


def _empty(*shape, dev):
    return torch.empty(*shape, device=dev, dtype=torch.float32)


# ------------------------------------------------------------------------------------------------
# Subsampling (A.3): im2col + MFMA GEMM, ReLU and frame masks fused into the epilogues.
# ------------------------------------------------------------------------------------------------

def _out_linear(cfg, S, P, pre, y, *, train, seed, salt, ws):
    """Linear(C*F -> d) on the channels-last (f, c) flattening of the last stage (weight re-laid
    out (d, F, C) on device), x*sqrt(d) and pre-encoder dropout fused."""
    d, C = S.d, S.C
    wout = ws["wout_perm"]
    K.convw_prep(P[pre + "pre_encode.out.weight"].view(d, C, S.F2), fwd=wout)
    xscale = math.sqrt(d) if cfg.xscaling else 1.0
    bscaled = ws["bout_scaled"]
    K.axpby(P[pre + "pre_encode.out.bias"].view(1, d), None, bscaled.view(1, d), alpha=xscale)
    x = _empty(S.rows, d, dev=y.device)
    p_pre = cfg.dropout_pre if train else 0.0
    K.linear(y.view(S.rows, S.F2 * C), wout.view(d, S.F2 * C), bscaled, x, alpha=xscale, dropout_p=p_pre,
             seed=seed, rng_stream=_stream(salt, -1, SITE_PRE))
    return x, p_pre, xscale


def _out_linear_backward(S, P, G, pre, ctx, dx, y, *, seed, salt, ws, bf16_out=False):
    """-> gradient wrt the last stage's pre-activation (relu'(y) applied: y is a ReLU output); bf16_out: as a
    bf16 tensor from one kdfm_ss_out_dgrad pass (the operand both conv2 gradients read)."""
    d, C = S.d, S.C
    dlin = _empty(S.rows, d, dev=dx.device)
    K.dropout(dx, dlin, ctx["p_pre"], ctx["xscale"], seed, _stream(salt, -1, SITE_PRE))
    Gout = ws["wout_perm_grad"]
    yv = y.view(S.rows, S.F2 * C)

    def out_wgrad():   # parameter gradients only: on the weight-gradient stream
        K.fill(Gout, 0.0)
        K.linear_dw(dlin, yv, Gout.view(d, S.F2 * C))
        K.convw_grad(Gout, G[pre + "pre_encode.out.weight"].view(d, C, S.F2))
        K.colsum(dlin, G[pre + "pre_encode.out.bias"])
    _side(out_wgrad, dlin, yv)
    if bf16_out:
        wt = ws["wout_t_bf16"]
        K.ss_out_wprep(ws["wout_perm"].view(d, S.F2 * C), wt)
        g = torch.empty(y.shape[0], C, device=dx.device, dtype=torch.bfloat16)
        K.ss_out_dgrad(dlin, wt, yv, g.view(S.rows, S.F2 * C))
        return g
    g = _empty(y.shape[0], C, dev=dx.device)
    K.linear_dx(dlin, ws["wout_perm"].view(d, S.F2 * C), g.view(S.rows, S.F2 * C), epi=_lib.EPI_DRELU,
                aux=y.view(S.rows, S.F2 * C))
    return g


def dw_subsampling_forward(cfg, S: EncoderShapes, P, pre, mel, mel_len, lens, *, train, seed, salt, save, ws):
    """ConvSubsampling 'dw_striding' (oracle/ver5.py subsampling_dw_striding): direct 3x3 stride-2
    kernels (csrc/dwsub.hip) for the first conv and the depthwise convs, kdfm_gemm for the pointwise
    1x1 convs (bias + ReLU + frame mask in the epilogue) and the output Linear."""
    dev = mel.device
    B, C = S.B, S.C
    m = cfg.subsampling_mask
    L = lambda s: (mel_len if s == 0 else lens[s - 1]) if m else None   # noqa: E731  (stage-s frame lengths)
    T1, F1 = S.stages[1]
    a = _empty(B * T1 * F1, C, dev=dev)
    K.dwsub_conv(mel, L(0), P[pre + "pre_encode.conv.0.weight"], P[pre + "pre_encode.conv.0.bias"], a, L(1),
                 B, S.Tm, cfg.nfilt, 1, C, T1, F1, S.pad, relu=True)
    acts, dws = [a], []
    for st in range(1, len(S.stages) - 1):
        i = 2 + 3 * (st - 1)
        (Ti, Fi), (To, Fo) = S.stages[st], S.stages[st + 1]
        q = _empty(B * To * Fo, C, dev=dev)
        K.dwsub_conv(a, L(st), P[pre + f"pre_encode.conv.{i}.weight"], P[pre + f"pre_encode.conv.{i}.bias"], q,
                     L(st + 1), B, Ti, Fi, C, C, To, Fo, S.pad, relu=False)
        a = _empty(B * To * Fo, C, dev=dev)
        K.linear(q, P[pre + f"pre_encode.conv.{i + 1}.weight"].view(C, C), P[pre + f"pre_encode.conv.{i + 1}.bias"],
                 a, epi=_lib.EPI_RELU, rowmask=(lens[st], To, Fo) if m else None)
        dws.append(q)
        acts.append(a)
    x, p_pre, xscale = _out_linear(cfg, S, P, pre, a, train=train, seed=seed, salt=salt, ws=ws)
    ctx = None
    if save:
        ctx = dict(acts=acts, dws=dws, p_pre=p_pre, xscale=xscale, mel=mel, mel_len=mel_len, lens=lens)
    return x, ctx


def dw_subsampling_backward(cfg, S: EncoderShapes, P, G, pre, ctx, dx, *, seed, salt, ws):
    B, C = S.B, S.C
    m = cfg.subsampling_mask
    lens, mel_len = ctx["lens"], ctx["mel_len"]
    L = lambda s: (mel_len if s == 0 else lens[s - 1]) if m else None   # noqa: E731
    acts, dws = ctx["acts"], ctx["dws"]
    g = _out_linear_backward(S, P, G, pre, ctx, dx, acts[-1], seed=seed, salt=salt, ws=ws)
    for st in range(len(S.stages) - 2, 0, -1):
        # g: gradient wrt the pre-activation of pointwise conv `st` (stage st+1 frames)
        i = 2 + 3 * (st - 1)
        (Ti, Fi), (To, Fo) = S.stages[st], S.stages[st + 1]
        q = dws[st - 1]
        Wpw = P[pre + f"pre_encode.conv.{i + 1}.weight"].view(C, C)
        WGRAD.run(lambda g=g, q=q, i=i: K.linear_dw(g, q, G[pre + f"pre_encode.conv.{i + 1}.weight"].view(C, C),
                                                    db=G[pre + f"pre_encode.conv.{i + 1}.bias"]), g, q)
        gq = _empty(B * To * Fo, C, dev=dx.device)
        K.linear_dx(g, Wpw, gq, rowmask=(lens[st], To, Fo) if m else None)
        a_in = acts[st - 1]
        K.dwsub_conv_wgrad(gq, L(st + 1), a_in, L(st), G[pre + f"pre_encode.conv.{i}.weight"],
                           G[pre + f"pre_encode.conv.{i}.bias"], B, Ti, Fi, C, C, To, Fo, S.pad)
        ga = _empty(B * Ti * Fi, C, dev=dx.device)
        K.dwsub_conv_dgrad(gq, L(st + 1), P[pre + f"pre_encode.conv.{i}.weight"], a_in, L(st), ga, B, Ti, Fi, C, To,
                           Fo, S.pad)
        g = ga
    T1, F1 = S.stages[1]
    K.dwsub_conv_wgrad(g, L(1), ctx["mel"], L(0), G[pre + "pre_encode.conv.0.weight"], G[pre + "pre_encode.conv.0.bias"],
                       B, S.Tm, cfg.nfilt, 1, C, T1, F1, S.pad)


# KDFM_SS_ONE_KERNEL=0: the two-kernel striding forward (conv1 to HBM, implicit-GEMM conv2) instead of the
# one-kernel form
_SS_ONE_KERNEL = __import__("os").environ.get("KDFM_SS_ONE_KERNEL", "1") == "1"
# KDFM_SS_WGRAD_GATHER=0: the conv2 weight gradient over an im2col column matrix instead of the direct gather
_SS_WGRAD_GATHER = __import__("os").environ.get("KDFM_SS_WGRAD_GATHER", "1") == "1"
# KDFM_SIDE_FOLDS=1: the LayerNorm / depthwise folds and the subsampling output's weight gradient go to the
# weight-gradient stream (=0, default: they stay on the compute stream -- measured 2111 / 2116 vs 2074 / 2095
# utt/s, profiles/r04/r4v: the extra launches there delay the compute stream's dispatch more than they save)
_SIDE_FOLDS = __import__("os").environ.get("KDFM_SIDE_FOLDS", "0") == "1"


def _side(fn, *keep):
    if _SIDE_FOLDS:
        WGRAD.run(fn, *keep)
    else:
        fn()


# KDFM_SS_Y1_PAD=0: the fused subsampling forward's bf16 y1 rows unpadded (C channels; A/B switch)
_SS_Y1_PAD = __import__("os").environ.get("KDFM_SS_Y1_PAD", "1") == "1"

# KDFM_BN_ON_LOAD=0: the BN-SiLU backward's elementwise half as its own launch (A/B switch)
_BN_ON_LOAD = __import__("os").environ.get("KDFM_BN_ON_LOAD", "1") == "1"


def subsampling_forward(cfg, S: EncoderShapes, P, pre, mel, mel_len, len1, len2, *, train, seed, salt, save, ws):
    if cfg.subsampling == "dw_striding":
        return dw_subsampling_forward(cfg, S, P, pre, mel, mel_len, len1, train=train, seed=seed, salt=salt,
                                      save=save, ws=ws)
    dev = mel.device
    B, C, d = S.B, S.d, S.d
    cols1 = y1 = None
    y2 = _empty(B * S.T * S.F2, C, dev=dev)
    m0 = mel_len if cfg.subsampling_mask else None
    m1 = len1 if cfg.subsampling_mask else None
    m2 = len2 if cfg.subsampling_mask else None
    if K.get_math() == "bf16" and _SS_ONE_KERNEL and "ss_fused_w" in ws and S.F2 * 4 == cfg.nfilt:
        # one kernel (csrc/ssfused.hip): conv1 computed per workgroup into LDS (MFMA over hi/lo bf16 splits),
        # conv2 as an implicit GEMM over it; y1 reaches HBM only as the trained student's bf16 side output
        # (the backward's ReLU' sign and conv2 weight-gradient columns)
        # y1 rows padded to whole 32-channel chunks (96 at C = 88; zeros past C): each chunk's stores are then
        # whole 64-byte segments instead of runs straddling the 176-byte rows (KDFM_SS_Y1_PAD=0: unpadded)
        ldy1 = -(-C // 32) * 32 if _SS_Y1_PAD else C
        y1b = torch.empty(B * S.T1 * S.F1, ldy1, device=dev, dtype=torch.bfloat16) if save else None
        wp = ws["ss_fused_w"]
        K.subsample_fused_wprep(P[pre + "pre_encode.conv.0.weight"], P[pre + "pre_encode.conv.2.weight"], wp)
        K.subsample_fused(mel, m0, m1, m2, wp, P[pre + "pre_encode.conv.0.bias"], P[pre + "pre_encode.conv.2.bias"],
                          y2, y1b, B, S.Tm, cfg.nfilt, C)
        y1 = y1b
        del y1b
    elif K.get_math() == "bf16" and C % 8 == 0 and C <= 192:
        # fused: direct conv1 (+ReLU+masks) -> bf16 y1, implicit-GEMM conv2 (+bias+ReLU+mask); no
        # im2col matrix.  The backward keeps the same bf16 y1: its ReLU' needs only the sign and the conv2
        # weight gradient's columns are bf16 anyway (an f32 copy would be 2x the bytes, written and re-read).
        y1b = torch.empty(B * S.T1 * S.F1, C, device=dev, dtype=torch.bfloat16)
        K.subsample_conv1(mel, m0, m1, P[pre + "pre_encode.conv.0.weight"], P[pre + "pre_encode.conv.0.bias"], y1b, None,
                          B, S.Tm, cfg.nfilt, C)
        wb = ws["w2_bf16"]
        K.subsample_wprep(P[pre + "pre_encode.conv.2.weight"], wb)
        K.subsample_conv2(y1b, m2, wb, P[pre + "pre_encode.conv.2.bias"], y2, B, S.T1, S.F1, C)
        y1 = y1b if save else None
        del y1b
    else:
        cols0 = _empty(B * S.T1 * S.F1, 9, dev=dev)
        K.im2col_3x3s2(mel, m0, cols0, B, S.Tm, cfg.nfilt, 1)
        y1 = _empty(B * S.T1 * S.F1, C, dev=dev)
        w0 = P[pre + "pre_encode.conv.0.weight"].view(C, 9)
        K.linear(cols0, w0, P[pre + "pre_encode.conv.0.bias"], y1, epi=_lib.EPI_RELU,
                 rowmask=(len1, S.T1, S.F1) if cfg.subsampling_mask else None, math="f32")
        del cols0   # the conv0 weight gradient reads the mel frames directly
        cols1 = _empty(B * S.T * S.F2, 9 * C, dev=dev)
        K.im2col_3x3s2(y1, m1, cols1, B, S.T1, S.F1, C)
        w2 = P[pre + "pre_encode.conv.2.weight"].view(C, 9 * C)
        K.linear(cols1, w2, P[pre + "pre_encode.conv.2.bias"], y2, epi=_lib.EPI_RELU,
                 rowmask=(len2, S.T, S.F2) if cfg.subsampling_mask else None)
        if not save:
            del cols1
            cols1 = None
    x, p_pre, xscale = _out_linear(cfg, S, P, pre, y2, train=train, seed=seed, salt=salt, ws=ws)
    ctx = None
    if save:
        ctx = dict(y1=y1, cols1=cols1, y2=y2, p_pre=p_pre, xscale=xscale, mel=mel, mel_len=mel_len)
    return x, ctx


def subsampling_backward(cfg, S: EncoderShapes, P, G, pre, ctx, dx, len1, *, seed, salt, ws):
    if cfg.subsampling == "dw_striding":
        return dw_subsampling_backward(cfg, S, P, G, pre, ctx, dx, seed=seed, salt=salt, ws=ws)
    dev = dx.device
    B, C = S.B, S.C
    direct = K.get_math() == "bf16" and K.subsample_dgrad_supported(C) and ctx["cols1"] is None
    # the direct path's conv2 gradients both read dy2 as bf16: the output Linear's backward writes it so
    # (kdfm_ss_out_dgrad) instead of an f32 dy2 plus a cast
    dy2h = None
    if direct and "wout_t_bf16" in ws and B * S.T1 * S.F1 < (1 << 24):
        dy2h = _out_linear_backward(S, P, G, pre, ctx, dx, ctx["y2"], seed=seed, salt=salt, ws=ws, bf16_out=True)
        dy2 = None
    else:
        dy2 = _out_linear_backward(S, P, G, pre, ctx, dx, ctx["y2"], seed=seed, salt=salt, ws=ws)
    if direct:
        # conv2 weight gradient on the weight-gradient stream from bf16 operands and the bf16 dy2, one
        # row-parallel launch into (C, 9, C) then re-laid out into (C, C, 3, 3): gathered straight from the
        # bf16 y1 (kdfm_wgrad_bf16_s2conv) when the fused forward kept it so, else over tap-major bf16
        # columns of y1 (KDFM_SS_WGRAD_GATHER=0: the column matrix, 9/4 x |y1| written and read back)
        y1 = ctx["y1"]
        gather = _SS_WGRAD_GATHER and y1.dtype == torch.bfloat16 and C % 8 == 0 and S.F1 >= 7
        cols1 = None if gather else torch.empty(B * S.T * S.F2, 9 * C, device=dev, dtype=torch.bfloat16)
        cast = dy2h is None
        if cast:
            dy2h = torch.empty(B * S.T * S.F2, C, device=dev, dtype=torch.bfloat16)
        gtm = ws["w2_tapmajor_grad"]
        lin = len1 if cfg.subsampling_mask else None

        def conv2_wgrad():
            if not gather:
                K.im2col_3x3s2_tm_bf16(y1, lin, cols1, B, S.T1, S.F1, C)
            if cast:
                K.cast_bf16(dy2, dy2h)
            K.fill(gtm, 0.0)
            if gather:
                K.wgrad_bf16_s2conv(dy2h, y1, lin, gtm.view(C, 9 * C), G[pre + "pre_encode.conv.2.bias"], B, S.T1,
                                    S.F1, C)
            else:
                K.wgrad_bf16(dy2h, cols1, gtm.view(C, 9 * C), db=G[pre + "pre_encode.conv.2.bias"])
            K.wgrad_fold_flush()   # gtm is read below (deferred folds, fold_arena)
            K.convw_grad(gtm.view(C, 9 * C), G[pre + "pre_encode.conv.2.weight"].view(C, C, 9))
        WGRAD.run(conv2_wgrad, *(t for t in (dy2, cols1, dy2h, y1, len1) if t is not None))
    else:
        if ctx["y1"] is not None and ctx["y1"].dtype == torch.bfloat16:   # fused forward kept only the bf16 y1
            ctx["y1"] = ctx["y1"][:, :C].float().contiguous()
        cols1 = ctx["cols1"]
        rebuild = cols1 is None
        if rebuild:   # fused forward: the im2col operand of the conv2 weight gradient is rebuilt on the
            cols1 = _empty(B * S.T * S.F2, 9 * C, dev=dev)   # weight-gradient stream, beside the data gradient

        def conv2_wgrad():
            if rebuild:
                K.im2col_3x3s2(ctx["y1"], len1 if cfg.subsampling_mask else None, cols1, B, S.T1, S.F1, C)
            K.linear_dw(dy2, cols1, G[pre + "pre_encode.conv.2.weight"].view(C, 9 * C),
                        db=G[pre + "pre_encode.conv.2.bias"])
        WGRAD.run(conv2_wgrad, dy2, cols1, ctx["y1"], len1)
    m = cfg.subsampling_mask
    if direct and B * S.T1 * S.F1 < (1 << 24):
        # direct transposed conv over the input positions' parity classes (no column matrix), the ReLU'
        # of y1 in its epilogue, and conv0's weight gradient accumulated from the mel patches in the same
        # epilogue: dy1 never reaches HBM
        wt = ws["w2_dgrad"]
        K.subsample_dgrad_wprep(P[pre + "pre_encode.conv.2.weight"].view(C, C, 3, 3), wt)
        if dy2 is None:
            K.subsample_conv2_dgrad_w0_h(dy2h, wt, ctx["y1"], B, S.T1, S.F1, C, ctx["mel"],
                                         ctx["mel_len"] if m else None, S.Tm, cfg.nfilt, S.pad,
                                         G[pre + "pre_encode.conv.0.weight"].view(C, 9), G[pre + "pre_encode.conv.0.bias"])
        else:
            K.subsample_conv2_dgrad_w0(dy2, wt, ctx["y1"], B, S.T1, S.F1, C, ctx["mel"], ctx["mel_len"] if m else None,
                                       S.Tm, cfg.nfilt, S.pad, G[pre + "pre_encode.conv.0.weight"].view(C, 9),
                                       G[pre + "pre_encode.conv.0.bias"])
        return
    dy1 = _empty(B * S.T1 * S.F1, C, dev=dev)
    if direct:
        # direct transposed conv over the input positions' parity classes (no column matrix); the
        # ReLU' of y1 (zero at masked frames) is applied in its epilogue
        wt = ws["w2_dgrad"]
        K.subsample_dgrad_wprep(P[pre + "pre_encode.conv.2.weight"].view(C, C, 3, 3), wt)
        K.subsample_conv2_dgrad(dy2, wt, ctx["y1"], dy1, B, S.T1, S.F1, C)
    else:
        # data gradient in TAP-MAJOR columns (tap*C + c): GEMM against the (C, 9, C) re-laid weight, so
        # the col2im gather reads contiguous channel runs per tap
        w2tm = ws["w2_tapmajor"]
        K.convw_prep(P[pre + "pre_encode.conv.2.weight"].view(C, C, 9), fwd=w2tm)
        dcols1 = _empty(B * S.T * S.F2, 9 * C, dev=dev)
        K.linear_dx(dy2, w2tm.view(C, 9 * C), dcols1)
        K.col2im_3x3s2(dcols1, len1 if cfg.subsampling_mask else None, ctx["y1"], dy1, B, S.T1, S.F1, C, tapmajor=True)
        del dcols1
    del dy2
    # conv0 (1 -> C, 3x3, s2) weight gradient straight from the mel frames: the direct stride-2 kernel
    # of dw_striding's first stage (same layer), no im2col of the input, deterministic fold
    run = (lambda fn, *keep: fn()) if direct else WGRAD.run   # direct: the main stream is free here
    # every tensor the side-stream launch reads stays referenced until the join (the frame lengths too: the
    # module API frees its autograd ctx right after this backward, and a 16-byte length block is the first
    # one the allocator hands out again)
    run(lambda: K.dwsub_conv_wgrad(dy1, len1 if m else None, ctx["mel"], ctx["mel_len"] if m else None,
                                         G[pre + "pre_encode.conv.0.weight"], G[pre + "pre_encode.conv.0.bias"],
                                         B, S.Tm, cfg.nfilt, 1, C, S.T1, S.F1, S.pad), dy1, ctx["mel"], len1,
        ctx["mel_len"])
    

# ------------------------------------------------------------------------------------------------
# One ConformerLayer
# ------------------------------------------------------------------------------------------------

def _ln(x, P, name, eps, dev, save_stats=True, bf16=False):
    """bf16: the LN output in bf16 -- for an output whose every consumer is a large-tile product (_ln_bf16), which
    reads bf16 operands: the same bits its cast of an f32 output gave, half the write and no cast per read."""
    rows, d = x.shape
    y = torch.empty(rows, d, device=dev, dtype=torch.bfloat16) if bf16 else _empty(rows, d, dev=dev)
    m = _empty(rows, dev=dev)
    r = _empty(rows, dev=dev)
    K.layernorm_fwd(x, P[name + ".weight"], P[name + ".bias"], y, m, r, eps)
    return y, m, r


# bf16 math: the fused macaron FFN block (csrc/ffn.hip) where the shape is supported (KDFM_FFN_FUSED=0: the
# LayerNorm + two-GEMM path; the f32 parity mode always takes it)
_FFN_FUSED = __import__("os").environ.get("KDFM_FFN_FUSED", "1") == "1"


def _lnproj_fused(kind, rows, d, save):
    """bf16 math: LN-fused q|k|v / pointwise-conv1+GLU kernels where compiled (KDFM_LNPROJ_FUSED=0: the
    LN + GEMM + prep path; training also needs the fused backward and the bf16 weight-gradient shape)."""
    if not (_LNPROJ_FUSED and K.get_math() == "bf16" and K.lnproj_supported(kind, d)):
        return False
    if not save:
        return True
    n = (3 if kind == K.LNPROJ_QKV else 2) * d
    return K.lnproj_supported(kind, d, bwd=True) and K.wgrad_bf16_supported(rows, n, d)


_LNPROJ_FUSED = __import__("os").environ.get("KDFM_LNPROJ_FUSED", "1") == "1"
_ROWGEMM_FUSED = __import__("os").environ.get("KDFM_ROWGEMM_FUSED", "1") == "1"


def _rowgemm_fused(rows, d, save):
    """bf16 math: the d x d products (linear_out, BN-SiLU + pointwise_conv2) on kdfm_rowgemm
    (KDFM_ROWGEMM_FUSED=0: kdfm_gemm + separate BN-SiLU / dropout kernels)."""
    if not (_ROWGEMM_FUSED and K.get_math() == "bf16" and K.rowgemm_supported(d)):
        return False
    return not save or K.wgrad_bf16_supported(rows, d, d)


def _ffn_forward(cfg, P, L, which, norm, x, pd, seed, salt, li, site_act, site_out, save, keep, tag, out_ln=None):
    """r_out = r_in + 0.5*drop(W2 drop(silu(W1 LN(r_in) + b1)) + b2) (NeMo ConformerFeedForward half step).
    out_ln = (norm name, y): the fused kernel also writes y = LN(r_out) (the layer's norm_out) and keeps
    its row statistics as m5 / r5; returns (r_out, True) then, else (r_out, False)."""
    rows, d = x.shape
    dev = x.device
    W1, W2 = P[L + which + ".linear1.weight"], P[L + which + ".linear2.weight"]
    ff = W1.shape[0]
    out = _empty(rows, d, dev=dev)
    if _FFN_FUSED and K.get_math() == "bf16" and K.ffn_supported(d, ff) and (
            not save or (K.wgrad_bf16_supported(rows, d, ff) and K.wgrad_bf16_supported(rows, ff, d))):
        m = _empty(rows, dev=dev) if save else None
        r = _empty(rows, dev=dev) if save else None
        img = K.ffn_img(W1, W2, fwd_only=not save)
        oln = None
        if out_ln is not None:
            m5, r5 = _empty(rows, dev=dev), _empty(rows, dev=dev)
            oln = (P[out_ln[0] + ".weight"], P[out_ln[0] + ".bias"], cfg.ln_eps, out_ln[1], m5, r5)
            keep(m5=m5, r5=r5)
        K.ffn_fwd(x, P[norm + ".weight"], P[norm + ".bias"], cfg.ln_eps, img, P[L + which + ".linear1.bias"],
                  P[L + which + ".linear2.bias"], out, m, r, ff, rscale=0.5, p_act=pd, p_out=pd, seed=seed,
                  st_act=_stream(salt, li, site_act), st_out=_stream(salt, li, site_out), out_ln=oln)
        keep(**{"m" + tag: m, "r" + tag: r, "ffn_img" + tag: img})
        return out, out_ln is not None
    ln, m, r = _ln(x, P, norm, cfg.ln_eps, dev, bf16=_ln_bf16(rows, d, ff, save))
    h = _empty(rows, ff, dev=dev) if save else None
    # the hidden activation in bf16 when its producer and every consumer take the large-tile route (d_model >= 512):
    # the values those products read are bf16-rounded anyway, so this halves its write and skips a cast per read
    bf_mid = _big_all((rows, ff, d, _lib.BIG_NT), (rows, d, ff, _lib.BIG_NT)) and (
        not save or _big_all((d, ff, rows, _lib.BIG_TN)))
    a = torch.empty(rows, ff, device=dev, dtype=torch.bfloat16) if bf_mid else _empty(rows, ff, dev=dev)
    K.linear(ln, W1, P[L + which + ".linear1.bias"], a, epi=_lib.EPI_SILU | (_lib.EPI_STORE_PRE if save else 0), Cpre=h,
             dropout_p=pd, seed=seed, rng_stream=_stream(salt, li, site_act), tag="ffn_up")
    K.linear(a, W2, P[L + which + ".linear2.bias"], out, epi=_lib.EPI_RESID, R=x, rscale=0.5, dropout_p=pd, seed=seed,
             rng_stream=_stream(salt, li, site_out))
    keep(**{"ln" + tag: ln, "m" + tag: m, "r" + tag: r, "h" + tag: h, "a" + tag: a})
    return out, False


def _big_all(*shapes):
    """Every (M, N, K, layout) product takes the large-tile bf16 route (kernels.big_ok)."""
    return all(K.big_ok(*sh) for sh in shapes)


def _grad_bf16(rows, n_out, k_in):
    """A Linear's output gradient (rows, n_out) can be produced in bf16: its data gradient (rows, k_in) and its
    weight gradient (n_out, k_in) both take the large-tile route, which reads bf16 operands anyway."""
    return _big_all((rows, k_in, n_out, _lib.BIG_NN), (n_out, k_in, rows, _lib.BIG_TN))


def _bf16_or_f32(use_bf16, rows, cols, dev):
    return torch.empty(rows, cols, device=dev, dtype=torch.bfloat16) if use_bf16 else _empty(rows, cols, dev=dev)


def _ln_bf16(rows, d, n, save):
    """The LN output feeding a (d -> n) projection can be bf16: the projection (and, training, its weight gradient)
    take the large-tile route, and the bf16 LN kernel applies."""
    return K.layernorm_bf16_ok(d) and _big_all((rows, n, d, _lib.BIG_NT)) and (
        not save or _big_all((n, d, rows, _lib.BIG_TN)))


def _fwd3_ok(dk, save):
    """The prepared-operand attention forward applies (bf16 fused attention, single pass)."""
    return _ATTN_FWD3 and _attn_fused_ok(dk, save) and (not save or (_ATTN_BWD_FUSED and _ATTN_BWD2))


def layer_forward(cfg, S: EncoderShapes, P, L, li, x, out, pos_emb, lengths, *, train, seed, salt, save,
                  bn_update=None, rm_batch=True, ppos=None, bn_stats=None, pband=None):
    """x (rows, d) -> out (rows, d) (written in place).  Returns ctx for backward when save.
    ppos: this layer's projected positions linear_pos(pos_emb) (npos, d) when the caller computed
    every layer's at once (pos_proj_all); otherwise projected here.  bn_stats: a zeroed (2d,) f64 buffer
    the BatchNorm batch sums may accumulate into when the training finalize runs (it leaves the buffer
    zeroed again, so the encoder's layers reuse one buffer without a memset per layer)."""
    dev = x.device
    rows, d, H, dk, T, B, ff = S.rows, S.d, S.h, S.dk, S.T, S.B, S.ff
    pd = cfg.dropout if train else 0.0
    pa = cfg.dropout_att if train else 0.0
    ctx = {} if save else None

    def keep(**kw):
        if save:
            ctx.update(kw)

    # ---- FFN1 (macaron half-step) ----
    x1, _ = _ffn_forward(cfg, P, L, "feed_forward1", L + "norm_feed_forward1", x, pd, seed, salt, li, SITE_FF1_ACT,
                         SITE_FF1_OUT, save, keep, "1")
    keep(x=x)

    # ---- relative-position MHSA ----
    qkv = _empty(rows, 3 * d, dev=dev)
    qu = _empty(rows, d, dev=dev)
    qv = _empty(rows, d, dev=dev)
    if _lnproj_fused(K.LNPROJ_QKV, rows, d, save):
        # LN + q|k|v projection + positional biases in one kernel (csrc/lnproj.hip); the backward
        # recomputes the bf16 LN output it needs for the weight gradient
        ln2 = None
        m2 = _empty(rows, dev=dev) if save else None
        r2 = _empty(rows, dev=dev) if save else None
        K.ln_qkv_fwd(x1, P[L + "norm_self_att.weight"], P[L + "norm_self_att.bias"], cfg.ln_eps,
                     K.lnproj_img(K.LNPROJ_QKV, P[L + "self_attn.qkv.weight"]), P[L + "self_attn.qkv.bias"],
                     P[L + "self_attn.pos_bias_u"], P[L + "self_attn.pos_bias_v"], qu, qv, qkv, m2, r2)
    else:
        ln2, m2, r2 = _ln(x1, P, L + "norm_self_att", cfg.ln_eps, dev, bf16=_ln_bf16(rows, d, 3 * d, save))
        K.linear(ln2, P[L + "self_attn.qkv.weight"], P[L + "self_attn.qkv.bias"], qkv)
        K.qkv_prep(qkv, P[L + "self_attn.pos_bias_u"], P[L + "self_attn.pos_bias_v"], qu, qv)
    npos = 2 * T - 1
    if ppos is None:
        ppos = _empty(npos, d, dev=dev)
        K.linear(pos_emb, P[L + "self_attn.linear_pos.weight"], None, ppos)
    o = _empty(rows, d, dev=dev)
    if _fwd3_ok(dk, save):
        # prepared operands: bf16 centred K / V tiles of this layer, the encoder's band rows (pband, or this
        # layer's own); lse for the bwd2 backward when training
        Pm = Pd = pt = mblk = None
        lse = torch.empty(B, H, T, device=dev) if save else None
        prep = K.attn_kv_prep(qkv, lengths, B, H, T)
        if pband is None:
            pband = K.attn_band_prep(ppos, H, T)[0]
        K.relpos_attn_fwd3(qu, qv, prep, pband, lengths, o, B, H, T, 1.0 / math.sqrt(dk), pa, seed,
                           _stream(salt, li, SITE_ATT_P), lse=lse)
        if save and _ATTN_DQ3:
            keep(attn_prep=prep, attn_pband=pband)
        del prep
    elif _attn_fused_ok(dk, save):
        # fused flash-style kernel: no AC / BD materialisation; P (and P_drop) only when the
        # backward needs them
        if _ATTN_BWD_FUSED:
            # one online-softmax pass; training keeps the per-row log-sum-exp (the backward's dQ kernel
            # recomputes P tile by tile from it) and the bf16 unnormalised p~ with its per-block maxima
            # (dK / dV and dPpos read P from them); dropout masks are regenerated from the counter RNG
            Pm = Pd = None
            if _ATTN_BWD2:
                lse, pt, mblk = (torch.empty(B, H, T, device=dev) if save else None), None, None
            else:
                lse, pt, mblk = K.attn_saved(B, H, T, dev) if save else (None, None, None)
        else:
            Pm = _empty(B, H, T, T, dev=dev) if save else None
            Pd = (_empty(B, H, T, T, dev=dev) if pa > 0 else Pm) if save else None
            lse = pt = mblk = None
        K.relpos_attn_fwd(qu, qv, qkv, ppos, lengths, o, Pm, Pd if pa > 0 else None, B, H, T,
                          1.0 / math.sqrt(dk), pa, seed, _stream(salt, li, SITE_ATT_P), lse=lse, p_tilde=pt, m_blk=mblk)
    else:
        ac = _empty(B, H, T, T, dev=dev)
        # AC = (q+u) K^T  per (b,h): A(i,c)=qu[b,i,h*dk+c]  B(c,j)=K[b,j,h*dk+c]
        K.gemm(qu, qkv[:, d:], ac, T, T, dk, d, 1, 1, 3 * d, T, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
               batch=(B, H), bA=(T * d, dk), bB=(T * 3 * d, dk), bC=(H * T * T, T * T))
        bd = _empty(B, H, T, npos, dev=dev)
        K.gemm(qv, ppos, bd, T, npos, dk, d, 1, 1, d, npos, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
               batch=(B, H), bA=(T * d, dk), bB=(0, dk), bC=(H * T * npos, T * npos))
        Pm = _empty(B, H, T, T, dev=dev)
        Pd = _empty(B, H, T, T, dev=dev) if pa > 0 else Pm
        K.relpos_softmax_fwd(ac, bd, lengths, Pm, Pd if pa > 0 else None, B, H, T, 1.0 / math.sqrt(dk), pa, seed,
                             _stream(salt, li, SITE_ATT_P))
        del ac, bd
        # O = Pd V : A = Pd (T x T), B(j,c) = V[b,j,h*dk+c]  -> o[b,i,h*dk+c]
        K.gemm(Pd, qkv[:, 2 * d:], o, T, dk, T, T, 1, 3 * d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
               batch=(B, H), bA=(H * T * T, T * T), bB=(T * 3 * d, dk), bC=(T * d, dk))
    x2 = _empty(rows, d, dev=dev)
    o_h = None
    if _rowgemm_fused(rows, d, save):
        # linear_out + dropout + residual on the row-streaming kernel; training keeps o as the bf16
        # weight-gradient operand it rounds anyway
        o_h = torch.empty(rows, d, device=dev, dtype=torch.bfloat16) if save else None
        K.rowgemm(o, K.rowgemm_img(P[L + "self_attn.linear_out.weight"]), x2, x_h=o_h, epi=K.RG_EPI_RESID,
                  bias=P[L + "self_attn.linear_out.bias"], R=x1, rscale=1.0, p_out=pd,
                  st_out=_stream(salt, li, SITE_ATT_OUT), seed=seed)
    else:
        o_in = o
        if _big_all((rows, d, d, _lib.BIG_NT)) and save and _big_all((d, d, rows, _lib.BIG_TN)):
            # linear_out and its weight gradient read bf16: one cast, kept for the backward (o itself stays f32 for
            # the attention backward's row sums)
            o_in = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
            K.cast_bf16(o, o_in)
            keep(o16=o_in)
        K.linear(o_in, P[L + "self_attn.linear_out.weight"], P[L + "self_attn.linear_out.bias"], x2, epi=_lib.EPI_RESID,
                 R=x1, rscale=1.0, dropout_p=pd, seed=seed, rng_stream=_stream(salt, li, SITE_ATT_OUT))
        del o_in
    fused_attn = _attn_fused_ok(dk, save) and _ATTN_BWD_FUSED
    keep(x1=x1, ln2=ln2, m2=m2, r2=r2, qkv=qkv, qu=qu, qv=qv, ppos=ppos, P=Pm, Pd=Pd, o=o, o_h=o_h, pa=pa,
         attn_fused=fused_attn, lse=lse if fused_attn else None, pt=pt if fused_attn else None,
         mblk=mblk if fused_attn else None)
    del ln2, qkv, qu, qv, ppos, Pm, Pd, o

    # ---- convolution module ----
    g = _empty(rows, d, dev=dev)
    if _lnproj_fused(K.LNPROJ_GLU, rows, d, save):
        # LN + pointwise_conv1 + GLU + pad mask in one kernel (csrc/lnproj.hip); the backward recomputes
        # the projection for GLU'
        ln3 = a = None
        m3 = _empty(rows, dev=dev) if save else None
        r3 = _empty(rows, dev=dev) if save else None
        K.ln_glu_fwd(x2, P[L + "norm_conv.weight"], P[L + "norm_conv.bias"], cfg.ln_eps,
                     K.lnproj_img(K.LNPROJ_GLU, P[L + "conv.pointwise_conv1.weight"].view(2 * d, d)),
                     P[L + "conv.pointwise_conv1.bias"], lengths, T, g, m3, r3)
    else:
        ln3, m3, r3 = _ln(x2, P, L + "norm_conv", cfg.ln_eps, dev, bf16=_ln_bf16(rows, d, 2 * d, save))
        a = _empty(rows, 2 * d, dev=dev)
        K.linear(ln3, P[L + "conv.pointwise_conv1.weight"].view(2 * d, d), P[L + "conv.pointwise_conv1.bias"], a)
        K.glu_mask_fwd(a, lengths, g, B, T, d)
    y = _empty(rows, d, dev=dev)
    fin_running = rm_batch and bn_update is not None and train
    bmean = _empty(d, dev=dev)
    brstd = _empty(d, dev=dev)
    rmn, rvr = bn_update if bn_update is not None else (None, None)
    if fin_running and bn_stats is not None:
        stats = bn_stats   # zero on entry; kdfm_bn_finalize_running re-zeroes it after reading
    else:
        stats = torch.zeros(2 * d, device=dev, dtype=torch.float64) if rm_batch else None
    with K.span("dwconv", nbytes=4.0 * 2 * rows * d):   # read g + write y (f32), SURVEY.md §8(d)
        K.dwconv_fwd(g, P[L + "conv.depthwise_conv.weight"].view(d, -1), P[L + "conv.depthwise_conv.bias"], y,
                     stats, B, T, d, cfg.conv_kernel)
    if stats is not None and rm_batch and bn_update is not None and train:
        # batch statistics and the running-statistics update in one launch
        K.bn_finalize_running(stats, rmn, rvr, bmean, brstd, d, rows, cfg.bn_eps, cfg.bn_momentum)
    else:
        K.bn_finalize(stats, rmn, rvr, bmean, brstd, d, rows, cfg.bn_eps)
        if rm_batch and bn_update is not None and train:
            K.bn_running_update(rmn, rvr, stats, d, rows, cfg.bn_momentum)
    x3 = _empty(rows, d, dev=dev)
    z = z_h = None
    if _rowgemm_fused(rows, d, save):
        # BatchNorm + SiLU as the prologue of pointwise_conv2 (+ dropout + residual): z never reaches HBM
        # in f32; training keeps its bf16 copy for the weight gradient
        z_h = torch.empty(rows, d, device=dev, dtype=torch.bfloat16) if save else None
        K.rowgemm(y, K.rowgemm_img(P[L + "conv.pointwise_conv2.weight"].view(d, d)), x3, pro=K.RG_PRO_BNSILU,
                  bn=(bmean, brstd, P[L + "conv.batch_norm.weight"], P[L + "conv.batch_norm.bias"]), x_h=z_h,
                  epi=K.RG_EPI_RESID, bias=P[L + "conv.pointwise_conv2.bias"], R=x2, rscale=1.0, p_out=pd,
                  st_out=_stream(salt, li, SITE_CONV_OUT), seed=seed)
    else:
        # z in bf16 when pointwise_conv2 and its weight gradient take the large-tile route (they read bf16)
        z = _bf16_or_f32(_big_all((rows, d, d, _lib.BIG_NT)) and (not save or _big_all((d, d, rows, _lib.BIG_TN))),
                         rows, d, dev)
        K.bn_silu_fwd(y, bmean, brstd, P[L + "conv.batch_norm.weight"], P[L + "conv.batch_norm.bias"], z)
        K.linear(z, P[L + "conv.pointwise_conv2.weight"].view(d, d), P[L + "conv.pointwise_conv2.bias"], x3,
                 epi=_lib.EPI_RESID, R=x2, rscale=1.0, dropout_p=pd, seed=seed,
                 rng_stream=_stream(salt, li, SITE_CONV_OUT))
    keep(x2=x2, ln3=ln3, m3=m3, r3=r3, a=a, g=g, y=y, bmean=bmean, brstd=brstd, z=z, z_h=z_h, rm_batch=rm_batch)
    del ln3, a, g, y, z

    # ---- FFN2 ----
    x4, ln_done = _ffn_forward(cfg, P, L, "feed_forward2", L + "norm_feed_forward2", x3, pd, seed, salt, li,
                               SITE_FF2_ACT, SITE_FF2_OUT, save, keep, "4", out_ln=(L + "norm_out", out))
    # ---- norm_out -> hooked layer output (fused into the FFN2 kernel's epilogue when it ran) ----
    if not ln_done:
        m5 = _empty(rows, dev=dev)
        r5 = _empty(rows, dev=dev)
        K.layernorm_fwd(x4, P[L + "norm_out.weight"], P[L + "norm_out.bias"], out, m5, r5, cfg.ln_eps)
        keep(m5=m5, r5=r5)
    keep(x3=x3, x4=x4, pd=pd)
    return ctx


class LnGrads:
    """The five LayerNorm backwards of one ConformerLayer write dgamma|dbeta block partials into
    slots of one buffer and fold them with ONE launch at the end of the layer (kdfm_ln_fold)."""

    def __init__(self, buf, rows, d):
        self.buf, self.rows, self.d = buf, rows, d
        self.n = K.layernorm_bwd_ws(rows, d)
        self.pending = []

    def bwd(self, dy, x, g, mean, rstd, dx, dg, db, dres=None, dy2=None):
        part = self.buf[len(self.pending)][: self.n]
        K.layernorm_bwd_part(dy, x, g, mean, rstd, dx, part, dres=dres, dy2=dy2)
        self.pending.append((part, dg, db))

    def reserve(self, dg, db):
        """A partial slot for a LayerNorm backward computed elsewhere (the fused FFN kernel)."""
        part = self.buf[len(self.pending)][: self.n]
        self.pending.append((part, dg, db))
        return part

    def fold(self):
        """On the weight-gradient stream (the partials are complete when it forks): the buffer must not be
        reused by the next layer before the join -- encoder_backward gives every layer its own."""
        if self.pending:
            pend, rows, d = self.pending, self.rows, self.d
            _side(lambda: K.ln_fold(pend, rows, d), self.buf)
            self.pending = []


def _wgrad_paired(pend, key, L, dY, X, wname, bname, G):
    """Issue a bf16 weight gradient on the weight-gradient stream, paired with a waiting same-shape one:
    the first of a pair is parked in `pend[key]`, the second launches both (kdfm_wgrad_bf16_pair)."""
    if pend is None or not _WGRAD_PAIRS:
        WGRAD.run(lambda: K.wgrad_bf16(dY, X, G[wname], db=G[bname]), dY, X)
        return
    if key not in pend:
        pend[key] = (dY, X, wname, bname)
        return
    dY0, X0, w0, b0 = pend.pop(key)
    WGRAD.run(lambda: K.wgrad_bf16_pair(dY0, X0, G[w0], G[b0], dY, X, G[wname], G[bname]), dY0, X0, dY, X)


def _wgrad_flush(pend, G):
    """Launch what is still parked (a pair whose partner took another path) as single products."""
    if pend:
        for dY, X, w, b in list(pend.values()):
            WGRAD.run(lambda dY=dY, X=X, w=w, b=b: K.wgrad_bf16(dY, X, G[w], db=G[b]), dY, X)
        pend.clear()


def _ffn_backward(P, G, L, which, dres_out, ctx, tag, x_in_ln, norm, pd, seed, salt, li, site_act, site_out, dev,
                  lng, pend=None):
    """Backward of r_out = r_in + 0.5*drop(W2 drop(silu(W1 LN(r_in)))) ; returns d r_in."""
    rows, d = dres_out.shape
    m, r = ctx["m" + tag], ctx["r" + tag]
    img = ctx.get("ffn_img" + tag)
    if img is not None:
        # fused kernel: hidden chunk recomputed from LN(r_in), data gradient + LN backward in one launch;
        # the bf16 operands it writes feed the row-parallel weight gradients on the wgrad stream
        ff = P[L + which + ".linear1.weight"].shape[0]
        bf = torch.bfloat16
        ln_h = torch.empty(rows, d, device=dev, dtype=bf)
        dl2_h = torch.empty(rows, d, device=dev, dtype=bf)
        a_h = torch.empty(rows, ff, device=dev, dtype=bf)
        dh_h = torch.empty(rows, ff, device=dev, dtype=bf)
        dx = _empty(rows, d, dev=dev)
        part = lng.reserve(G[norm + ".weight"], G[norm + ".bias"])
        K.ffn_bwd(dres_out, x_in_ln, m, r, P[norm + ".weight"], P[norm + ".bias"], img,
                  P[L + which + ".linear1.bias"], dx, ln_h, a_h, dl2_h, dh_h, part, ff, rscale=0.5, p_act=pd, p_out=pd,
                  seed=seed, st_act=_stream(salt, li, site_act), st_out=_stream(salt, li, site_out))
        _wgrad_paired(pend, "ffn_l2", L, dl2_h, a_h, L + which + ".linear2.weight", L + which + ".linear2.bias", G)
        _wgrad_paired(pend, "ffn_l1", L, dh_h, ln_h, L + which + ".linear1.weight", L + which + ".linear1.bias", G)
        return dx
    ln, h, a = ctx["ln" + tag], ctx["h" + tag], ctx["a" + tag]
    ff = h.shape[1]
    dlin2 = _bf16_or_f32(_grad_bf16(rows, d, ff), rows, d, dev)
    K.dropout(dres_out, dlin2, pd, 0.5, seed, _stream(salt, li, site_out))
    WGRAD.run(lambda: K.linear_dw(dlin2, a, G[L + which + ".linear2.weight"], db=G[L + which + ".linear2.bias"]), dlin2, a)
    # the hidden gradient in bf16 when its producer and both consumers take the large-tile route (as `a` above)
    bf_mid = _big_all((rows, ff, d, _lib.BIG_NN), (rows, d, ff, _lib.BIG_NN), (ff, d, rows, _lib.BIG_TN))
    dh = torch.empty(rows, ff, device=dev, dtype=torch.bfloat16) if bf_mid else _empty(rows, ff, dev=dev)
    K.linear_dx(dlin2, P[L + which + ".linear2.weight"], dh, epi=_lib.EPI_DSILU, aux=h, dropout_p=pd, seed=seed,
                rng_stream=_stream(salt, li, site_act))
    del dlin2
    WGRAD.run(lambda: K.linear_dw(dh, ln, G[L + which + ".linear1.weight"], db=G[L + which + ".linear1.bias"]), dh, ln)
    dln = _empty(rows, d, dev=dev)
    K.linear_dx(dh, P[L + which + ".linear1.weight"], dln)
    del dh
    dx = _empty(rows, d, dev=dev)
    lng.bwd(dln, x_in_ln, P[norm + ".weight"], m, r, dx, G[norm + ".weight"], G[norm + ".bias"], dres=dres_out)
    return dx


def layer_backward(cfg, S: EncoderShapes, P, G, L, li, ctx, dout, pos_emb, lengths, *, seed, salt, ln_buf=None,
                   dout2=None, bn_red=None):
    """dout (+ dout2 when given): grad wrt the layer output (rows, d). Returns grad wrt the layer input.
    bn_red: (red, red_next) f64 (2d,) buffers of a ring: red zero on entry, red_next zeroed for the next
    layer (no memset launch per layer); None: a fresh buffer zeroed by the launch."""
    dev = dout.device
    rows, d, H, dk, T, B = S.rows, S.d, S.h, S.dk, S.T, S.B
    pd = ctx["pd"]
    if ln_buf is None:
        ln_buf = torch.empty(6, K.layernorm_bwd_ws(rows, d), device=dev)
    lng = LnGrads(ln_buf, rows, d)
    pend = ctx["_pend"] = {}   # same-shape bf16 weight gradients waiting for their pair (_wgrad_paired)
    # norm_out
    dx4 = _empty(rows, d, dev=dev)
    lng.bwd(dout, ctx["x4"], P[L + "norm_out.weight"], ctx["m5"], ctx["r5"], dx4, G[L + "norm_out.weight"],
            G[L + "norm_out.bias"], dy2=dout2)
    # FFN2: x4 = x3 + 0.5 drop(ffn(LN4 x3))
    dx3 = _ffn_backward(P, G, L, "feed_forward2", dx4, ctx, "4", ctx["x3"], L + "norm_feed_forward2", pd, seed, salt,
                        li, SITE_FF2_ACT, SITE_FF2_OUT, dev, lng, pend)
    del dx4
    # conv module: x3 = x2 + drop(pw2(z))
    dz = _empty(rows, d, dev=dev)
    if ctx.get("z_h") is not None:   # dropout prologue + data gradient on the row-streaming kernel
        dpw2_h = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
        K.rowgemm(dx3, K.rowgemm_img(P[L + "conv.pointwise_conv2.weight"].view(d, d), trans=True), dz,
                  pro=K.RG_PRO_DROP, p_in=pd, s_in=1.0, st_in=_stream(salt, li, SITE_CONV_OUT), x_h=dpw2_h, seed=seed)
        if _WGRAD_PAIRS:   # paired with linear_out's (same (d, d) shape) in the attention backward below
            pend["dd"] = (dpw2_h, ctx["z_h"], G[L + "conv.pointwise_conv2.weight"].view(d, d),
                          G[L + "conv.pointwise_conv2.bias"])
        else:
            WGRAD.run(lambda: K.wgrad_bf16(dpw2_h, ctx["z_h"], G[L + "conv.pointwise_conv2.weight"].view(d, d),
                                           db=G[L + "conv.pointwise_conv2.bias"]), dpw2_h, ctx["z_h"])
    else:
        dpw2 = _bf16_or_f32(_grad_bf16(rows, d, d), rows, d, dev)
        K.dropout(dx3, dpw2, pd, 1.0, seed, _stream(salt, li, SITE_CONV_OUT))
        WGRAD.run(lambda: K.linear_dw(dpw2, ctx["z"], G[L + "conv.pointwise_conv2.weight"].view(d, d), db=G[L + "conv.pointwise_conv2.bias"]), dpw2, ctx["z"])
        K.linear_dx(dpw2, P[L + "conv.pointwise_conv2.weight"].view(d, d), dz)
        del dpw2
    dg = _empty(rows, d, dev=dev)
    # the depthwise weight / bias gradient's fold of per-block partials runs on the weight-gradient stream
    dws = torch.empty(K.dwconv_bwd_ws(B, T, d, cfg.conv_kernel), device=dev)
    if _BN_ON_LOAD and bn_red is not None and cfg.conv_kernel in (9, 15, 31):
        # BN + SiLU backward: the sums, then their elementwise half applied on load by the depthwise backward
        # (dy never stored); the sums' buffer comes from the ring, the launch zeroes the next one
        Pbw, Pbb = P[L + "conv.batch_norm.weight"], P[L + "conv.batch_norm.bias"]
        K.bn_silu_bwd_reduce(dz, ctx["y"], ctx["bmean"], ctx["brstd"], Pbw, Pbb, bn_red[0])
        K.dwconv_bwd_bn(dz, ctx["y"], ctx["bmean"], ctx["brstd"], Pbw, Pbb, bn_red[0], bn_red[1],
                        G[L + "conv.batch_norm.weight"], G[L + "conv.batch_norm.bias"], ctx["rm_batch"], ctx["g"],
                        P[L + "conv.depthwise_conv.weight"].view(d, -1), dg, dws, B, T, d, cfg.conv_kernel)
        del dz
    else:
        dy = _empty(rows, d, dev=dev)
        if bn_red is not None:
            K.bn_silu_bwd(dz, ctx["y"], ctx["bmean"], ctx["brstd"], P[L + "conv.batch_norm.weight"],
                          P[L + "conv.batch_norm.bias"], bn_red[0], dy, G[L + "conv.batch_norm.weight"],
                          G[L + "conv.batch_norm.bias"], batch_stats=ctx["rm_batch"], red_next=bn_red[1],
                          zeroed=True)
        else:
            red = torch.empty(2 * d, device=dev, dtype=torch.float64)
            K.bn_silu_bwd(dz, ctx["y"], ctx["bmean"], ctx["brstd"], P[L + "conv.batch_norm.weight"],
                          P[L + "conv.batch_norm.bias"], red, dy, G[L + "conv.batch_norm.weight"],
                          G[L + "conv.batch_norm.bias"], batch_stats=ctx["rm_batch"])
        del dz
        K.dwconv_bwd(dy, ctx["g"], P[L + "conv.depthwise_conv.weight"].view(d, -1), dg, None, None, B, T, d,
                     cfg.conv_kernel, ws=dws)
        del dy
    _side(lambda: K.dwconv_bwd_fold(dws, G[L + "conv.depthwise_conv.weight"].view(d, -1),
                                    G[L + "conv.depthwise_conv.bias"], B, T, d, cfg.conv_kernel), dws)
    dx2 = _empty(rows, d, dev=dev)
    if ctx["ln3"] is None:   # fused LN + pointwise_conv1 + GLU forward: fused backward
        W1 = P[L + "conv.pointwise_conv1.weight"].view(2 * d, d)
        ln3_h = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
        da_h = torch.empty(rows, 2 * d, device=dev, dtype=torch.bfloat16)
        part = lng.reserve(G[L + "norm_conv.weight"], G[L + "norm_conv.bias"])
        K.ln_glu_bwd(dg, ctx["x2"], ctx["m3"], ctx["r3"], P[L + "norm_conv.weight"], P[L + "norm_conv.bias"],
                     K.lnproj_img(K.LNPROJ_GLU, W1, bwd=True), P[L + "conv.pointwise_conv1.bias"], lengths, T, dx3,
                     dx2, ln3_h, da_h, part)
        del dg, dx3
        WGRAD.run(lambda: K.wgrad_bf16(da_h, ln3_h, G[L + "conv.pointwise_conv1.weight"].view(2 * d, d),
                                       db=G[L + "conv.pointwise_conv1.bias"]), da_h, ln3_h)
    else:
        da = _bf16_or_f32(_grad_bf16(rows, 2 * d, d), rows, 2 * d, dev)
        K.glu_mask_bwd(dg, ctx["a"], lengths, da, B, T, d)
        del dg
        WGRAD.run(lambda: K.linear_dw(da, ctx["ln3"], G[L + "conv.pointwise_conv1.weight"].view(2 * d, d), db=G[L + "conv.pointwise_conv1.bias"]), da, ctx["ln3"])
        dln3 = _empty(rows, d, dev=dev)
        K.linear_dx(da, P[L + "conv.pointwise_conv1.weight"].view(2 * d, d), dln3)
        del da
        lng.bwd(dln3, ctx["x2"], P[L + "norm_conv.weight"], ctx["m3"], ctx["r3"], dx2, G[L + "norm_conv.weight"],
                G[L + "norm_conv.bias"], dres=dx3)
        del dln3, dx3
    # MHSA: x2 = x1 + drop(out(O))
    do = _empty(rows, d, dev=dev)
    if ctx.get("o_h") is not None:
        dlo_h = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
        K.rowgemm(dx2, K.rowgemm_img(P[L + "self_attn.linear_out.weight"], trans=True), do, pro=K.RG_PRO_DROP,
                  p_in=pd, s_in=1.0, st_in=_stream(salt, li, SITE_ATT_OUT), x_h=dlo_h, seed=seed)
        if "dd" in pend:
            dpw2_h, z_h, gw2, gb2 = pend.pop("dd")
            WGRAD.run(lambda: K.wgrad_bf16_pair(dpw2_h, z_h, gw2, gb2, dlo_h, ctx["o_h"],
                                                G[L + "self_attn.linear_out.weight"], G[L + "self_attn.linear_out.bias"]),
                      dpw2_h, z_h, dlo_h, ctx["o_h"])
        else:
            WGRAD.run(lambda: K.wgrad_bf16(dlo_h, ctx["o_h"], G[L + "self_attn.linear_out.weight"],
                                           db=G[L + "self_attn.linear_out.bias"]), dlo_h, ctx["o_h"])
    else:
        dlo = _bf16_or_f32(_grad_bf16(rows, d, d), rows, d, dev)
        K.dropout(dx2, dlo, pd, 1.0, seed, _stream(salt, li, SITE_ATT_OUT))
        o_w = ctx.get("o16") if ctx.get("o16") is not None else ctx["o"]
        WGRAD.run(lambda: K.linear_dw(dlo, o_w, G[L + "self_attn.linear_out.weight"], db=G[L + "self_attn.linear_out.bias"]), dlo, o_w)
        K.linear_dx(dlo, P[L + "self_attn.linear_out.weight"], do)
        del dlo
    qkv, Pm, Pd, qu, qv, ppos = ctx["qkv"], ctx["P"], ctx["Pd"], ctx["qu"], ctx["qv"], ctx["ppos"]
    npos = 2 * T - 1
    if ctx.get("attn_fused"):
        dqkv = _empty(rows, 3 * d, dev=dev)
        dqu = _empty(rows, d, dev=dev)
        dqv = _empty(rows, d, dev=dev)
        dppos = _empty(npos, d, dev=dev)
        sc = 1.0 / math.sqrt(dk)
        st_att = _stream(salt, li, SITE_ATT_P)
        # the positional-term gradient dPpos feeds only the linear_pos weight gradient: it runs on the
        # weight-gradient stream beside the dQ / dK,dV kernels the main stream needs next
        lse, pt, mblk = ctx["lse"], ctx["pt"], ctx["mblk"]
        if pt is None:   # bwd2
            dS, Pdr = K.attn_bwd2_saved(B, H, T, dev)
            prep = ctx.pop("attn_prep", None)
            if prep is not None:   # the forward's prepared bf16 operands (fwd3)
                K.relpos_attn_bwd2_dq3(do, ctx["o"], qu, qv, prep, ctx.pop("attn_pband"), lse, lengths, dS, Pdr, dqu, dqv,
                                       B, H, T, sc, ctx["pa"], seed, st_att)
                del prep
            else:
                K.relpos_attn_bwd2_dq(do, ctx["o"], qu, qv, qkv, ppos, lse, lengths, None, dS, Pdr, dqu, dqv, B, H, T,
                                      sc, ctx["pa"], seed, st_att)
            dpws = torch.empty(K.relpos_attn_bwd2_dpos_ws(B, T, d), device=dev)

            def dpos_and_wgrad2():
                K.relpos_attn_bwd2_dpos(qv, dS, lengths, dppos, B, H, T, ws=dpws)
                K.linear_dw(dppos, pos_emb, G[L + "self_attn.linear_pos.weight"])
            WGRAD.run(dpos_and_wgrad2, qv, dS, dppos, dpws, pos_emb, lengths)
            K.relpos_attn_bwd2_dkv(do, qu, dS, Pdr, lengths, dqkv, B, H, T)
            del do, Pdr, dS
            return _attn_bwd_tail(P, G, L, ctx, dqkv, dqu, dqv, None, pos_emb, dx2, lng, cfg, pd, seed, salt, li, rows,
                                  d, dev)
        abws = torch.empty(K.relpos_attn_bwd_ws(B, H, T, d), device=dev)
        K.relpos_attn_bwd(do, ctx["o"], qu, qv, qkv, ppos, lse, pt, mblk, lengths, dqu, dqv, dqkv, None, B, H, T, sc,
                          ctx["pa"], seed, st_att, parts=K.ATTN_BWD_ROWDOT | K.ATTN_BWD_DQ | K.ATTN_BWD_DKV, ws=abws)
        o_ = ctx["o"]

        def dpos_and_wgrad():
            K.relpos_attn_bwd(do, o_, qu, qv, qkv, ppos, lse, pt, mblk, lengths, None, None, None, dppos, B, H, T, sc,
                              ctx["pa"], seed, st_att, parts=K.ATTN_BWD_DPOS, ws=abws)
            K.linear_dw(dppos, pos_emb, G[L + "self_attn.linear_pos.weight"])
        WGRAD.run(dpos_and_wgrad, do, o_, qu, qv, qkv, ppos, lse, pt, mblk, dppos, abws, pos_emb, lengths, seed)
        del do
        return _attn_bwd_tail(P, G, L, ctx, dqkv, dqu, dqv, None, pos_emb, dx2, lng, cfg, pd, seed, salt, li, rows, d,
                              dev)
    dPd = _empty(B, H, T, T, dev=dev)
    # dPd = dO V^T : A(i,c)=do[b,i,h*dk+c], B(c,j)=V[b,j,h*dk+c]
    K.gemm(do, qkv[:, 2 * d:], dPd, T, T, dk, d, 1, 1, 3 * d, T, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
           batch=(B, H), bA=(T * d, dk), bB=(T * 3 * d, dk), bC=(H * T * T, T * T))
    dac = _empty(B, H, T, T, dev=dev)
    dbd = _empty(B, H, T, npos, dev=dev)
    K.relpos_softmax_bwd(Pm, dPd, dac, dbd, B, H, T, 1.0 / math.sqrt(dk), ctx["pa"], seed,
                         _stream(salt, li, SITE_ATT_P))
    del dPd
    dqkv = _empty(rows, 3 * d, dev=dev)
    # dV = Pd^T dO : A(j,i) = Pd[i,j] (XC), B(i,c) = do[b,i,h*dk+c] (XC) -> dqkv[b,j,2d+h*dk+c]
    K.gemm(Pd, do, dqkv[:, 2 * d:], T, dk, T, 1, T, d, 1, 3 * d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * d, dk), bC=(T * 3 * d, dk))
    del do
    dqu = _empty(rows, d, dev=dev)
    # dQu = dAC K : A = dac (KC), B(j,c) = K[b,j,h*dk+c] (XC)
    K.gemm(dac, qkv[:, d:], dqu, T, dk, T, T, 1, 3 * d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * 3 * d, dk), bC=(T * d, dk))
    # dK = dAC^T Qu : A(j,i) = dac[i,j] (XC), B(i,c) = qu (XC) -> dqkv[b,j,d+h*dk+c]
    K.gemm(dac, qu, dqkv[:, d:], T, dk, T, 1, T, d, 1, 3 * d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * d, dk), bC=(T * 3 * d, dk))
    del dac
    dqv = _empty(rows, d, dev=dev)
    # dQv = dBD Ppos : A = dbd (KC, T x npos), B(p,c) = ppos[p, h*dk+c] (XC)
    K.gemm(dbd, ppos, dqv, T, dk, npos, npos, 1, d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * npos, T * npos), bB=(0, dk), bC=(T * d, dk))
    dppos = torch.zeros(npos, d, device=dev)
    # dPpos[p, h*dk+c] += sum_b sum_i dbd[b,h,i,p] qv[b,i,h*dk+c]
    K.gemm(dbd, qv, dppos, npos, dk, T, 1, npos, d, 1, d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * npos, T * npos), bB=(T * d, dk), bC=(0, dk), epi=_lib.EPI_ATOMIC)
    del dbd
    return _attn_bwd_tail(P, G, L, ctx, dqkv, dqu, dqv, dppos, pos_emb, dx2, lng, cfg, pd, seed, salt, li, rows, d, dev)


def _attn_bwd_tail(P, G, L, ctx, dqkv, dqu, dqv, dppos, pos_emb, dx2, lng, cfg, pd, seed, salt, li, rows, d, dev):
    """Pos-bias / linear_pos / q|k|v projection grads, norm_self_att and FFN1 backward."""
    if dppos is not None:   # (the fused path ran dPpos and this weight gradient on the wgrad stream)
        WGRAD.run(lambda: K.linear_dw(dppos, pos_emb, G[L + "self_attn.linear_pos.weight"]), dppos, pos_emb)
    del dppos
    dx1 = _empty(rows, d, dev=dev)
    if ctx["ln2"] is None:   # fused LN + q|k|v forward: fused backward (dq = dqu + dqv formed in-kernel)
        ln2_h = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
        dqkv_h = torch.empty(rows, 3 * d, device=dev, dtype=torch.bfloat16)
        part = lng.reserve(G[L + "norm_self_att.weight"], G[L + "norm_self_att.bias"])
        # the positional-bias gradients ride along as one more partial entry of the layer's LN fold
        part_uv = lng.reserve(G[L + "self_attn.pos_bias_u"].view(-1), G[L + "self_attn.pos_bias_v"].view(-1))
        K.ln_qkv_bwd(dqu, dqv, dqkv, ctx["x1"], ctx["m2"], ctx["r2"], P[L + "norm_self_att.weight"],
                     P[L + "norm_self_att.bias"], K.lnproj_img(K.LNPROJ_QKV, P[L + "self_attn.qkv.weight"], bwd=True),
                     dx2, dx1, ln2_h, dqkv_h, part, part_uv)
        del dqu, dqv, dqkv, dx2
        WGRAD.run(lambda: K.wgrad_bf16(dqkv_h, ln2_h, G[L + "self_attn.qkv.weight"], db=G[L + "self_attn.qkv.bias"]),
                  dqkv_h, ln2_h)
    else:
        K.colsum(dqu, G[L + "self_attn.pos_bias_u"].view(-1))
        K.colsum(dqv, G[L + "self_attn.pos_bias_v"].view(-1))
        K.axpby(dqu, dqv, dqkv[:, :d], 1.0, 1.0)
        del dqu, dqv
        if _grad_bf16(rows, 3 * d, d):   # both consumers read bf16: one cast instead of one per consumer
            dq16 = torch.empty(rows, 3 * d, device=dev, dtype=torch.bfloat16)
            K.cast_bf16(dqkv, dq16)
            dqkv = dq16
            del dq16
        WGRAD.run(lambda: K.linear_dw(dqkv, ctx["ln2"], G[L + "self_attn.qkv.weight"], db=G[L + "self_attn.qkv.bias"]), dqkv, ctx["ln2"])
        dln2 = _empty(rows, d, dev=dev)
        K.linear_dx(dqkv, P[L + "self_attn.qkv.weight"], dln2)
        del dqkv
        lng.bwd(dln2, ctx["x1"], P[L + "norm_self_att.weight"], ctx["m2"], ctx["r2"], dx1,
                G[L + "norm_self_att.weight"], G[L + "norm_self_att.bias"], dres=dx2)
        del dln2, dx2
    # FFN1
    pend = ctx.pop("_pend", None)
    if pend and "dd" in pend:   # linear_out took the unfused path: pointwise_conv2's gradient alone
        dpw2_h, z_h, gw2, gb2 = pend.pop("dd")
        WGRAD.run(lambda: K.wgrad_bf16(dpw2_h, z_h, gw2, db=gb2), dpw2_h, z_h)
    dx = _ffn_backward(P, G, L, "feed_forward1", dx1, ctx, "1", ctx["x"], L + "norm_feed_forward1", pd, seed, salt, li,
                       SITE_FF1_ACT, SITE_FF1_OUT, dev, lng, pend)
    if pend:
        _wgrad_flush(pend, G)
    lng.fold()   # the layer's five dgamma/dbeta folds in one launch
    return dx


# ------------------------------------------------------------------------------------------------
# Whole encoder
# ------------------------------------------------------------------------------------------------

class EncoderRun:
    """Forward state of one encoder pass (what backward needs)."""

    def __init__(self):
        self.sub = None
        self.layers = []


_PP_BUF = {}


def pos_proj_all(cfg, P, prefix, pos_emb):
    """Every layer's linear_pos(pos_emb) in ONE batched GEMM -> (n_layers, npos, d), or None.

    The projection depends only on the (fixed) relative positions and each layer's weight, so the
    encoder computes all of them before its first layer instead of one small (npos x d x d) launch per
    layer on the critical stream (the reference applies NeMo's RelPositionMultiHeadAttention.linear_pos
    inside every layer).  Needs the layers' weights at one element stride (the flat parameter buffer);
    anything else, or KDFM_POS_BATCH=0, keeps the per-layer projection."""
    nl = cfg.n_layers
    if nl < 2 or os.environ.get("KDFM_POS_BATCH", "1") == "0":
        return None
    Ws = [P[f"{prefix}layers.{i}.self_attn.linear_pos.weight"] for i in range(nl)]
    d = Ws[0].shape[0]
    es = Ws[0].element_size()
    st = (Ws[1].data_ptr() - Ws[0].data_ptr()) // es
    if st <= 0 or any(W.shape != (d, d) or W.stride() != (d, 1) or W.dtype != torch.float32 or
                      W.data_ptr() - Ws[0].data_ptr() != i * st * es for i, W in enumerate(Ws)):
        return None
    npos = pos_emb.shape[0]
    # one persistent buffer per weight set: a per-step allocation freed while another stream's layers
    # still read it breaks the stream-ordered reuse of torch's pools (the eager step then differed from
    # its recorded plan); the next step's projection is ordered after every reader of this one (the
    # step's streams join before the optimizer, and the teacher stream waits for the main stream)
    key = (Ws[0].data_ptr(), st, nl, npos, d, pos_emb.device)
    out = _PP_BUF.get(key)
    if out is None:
        out = _PP_BUF[key] = _empty(nl, npos, d, dev=pos_emb.device)
    # out[l] = pos_emb @ W_l^T : A = pos_emb (KC), B(k, n) = W_l[n][k] (KC), batch l over W and out
    K.gemm(pos_emb, Ws[0], out, npos, d, d, pos_emb.stride(0), pos_emb.stride(1), 1, d, d, 1,
           amode=_lib.LD_KC, bmode=_lib.LD_KC, batch=(nl, 1), bA=(0, 0), bB=(st, 0), bC=(npos * d, 0))
    return out


def encoder_forward_steps(cfg, S: EncoderShapes, P, prefix, mel, mel_len, len1, len2, feats, pos_emb, *, train,
                          seed, salt, save, bn_running=None, use_batch_stats=True, ws, run=None):
    """Generator form of encoder_forward: issues the subsampling, then one layer per next() (the
    engine interleaves the teacher's and the student's launches this way, so both HIP streams get
    work from the first microsecond instead of one encoder waiting for the host to issue the other).
    `run` (an EncoderRun, when save) is filled as it goes."""
    x, sctx = subsampling_forward(cfg, S, P, prefix, mel, mel_len, len1, len2, train=train, seed=seed, salt=salt,
                                  save=save, ws=ws)
    if save:
        run.sub = sctx
    yield
    # after the yield: the caller issues the layers under their own stream, and the projections must be
    # allocated (torch's per-stream pools) and written on the stream whose layers read them
    pp = pos_proj_all(cfg, P, prefix, pos_emb)
    # every layer's positional band rows for the prepared-operand attention forward in one launch
    pbands = K.attn_band_prep(pp, S.h, S.T) if (pp is not None and _fwd3_ok(S.dk, save)) else None
    bn_stats = None
    if train and bn_running is not None and use_batch_stats:
        bn_stats = ws.get("bn_stats")
        if bn_stats is None:
            bn_stats = ws["bn_stats"] = torch.zeros(2 * S.d, device=mel.device, dtype=torch.float64)
    for i in range(cfg.n_layers):
        L = f"{prefix}layers.{i}."
        bn = None
        if bn_running is not None:
            bn = (bn_running[L + "conv.batch_norm.running_mean"], bn_running[L + "conv.batch_norm.running_var"])
        ctx = layer_forward(cfg, S, P, L, i, x, feats[i], pos_emb, len2, train=train, seed=seed, salt=salt,
                            save=save, bn_update=bn, rm_batch=use_batch_stats, ppos=None if pp is None else pp[i],
                            bn_stats=bn_stats, pband=None if pbands is None else pbands[i])
        if save:
            run.layers.append(ctx)
        x = feats[i]
        yield


def encoder_forward(cfg, S: EncoderShapes, P, prefix, mel, mel_len, len1, len2, feats, pos_emb, *, train, seed,
                    salt, save, bn_running=None, use_batch_stats=True, ws):
    """mel (B, Tm, nfilt) -> feats (n_layers, rows, d) filled; returns EncoderRun when save."""
    run = EncoderRun() if save else None
    for _ in encoder_forward_steps(cfg, S, P, prefix, mel, mel_len, len1, len2, feats, pos_emb, train=train, seed=seed,
                                   salt=salt, save=save, bn_running=bn_running, use_batch_stats=use_batch_stats,
                                   ws=ws, run=run):
        pass
    return run


def fold_arena(ws, dev):
    """The deferred weight-gradient folds' partial arena of an encoder workspace (bf16 math, KDFM_FOLD_DEFER).
    Sized _FOLD_ARENA_FLOATS, or -- when the previous backward had products that did not fit and folded at once
    (silent fallbacks at the XL shapes) -- the largest demand the library counted between two flushes.
    A replaced arena is only ever dropped between steps; a recorded step plan keeps the one it addresses
    (Ver5Engine.make_plan)."""
    if not _FOLD_DEFER or K.get_math() != "bf16":
        return None
    arena = ws.get("fold_arena")
    st = ws.pop("fold_stats", None)
    if arena is not None and st is not None and st[1] > 0 and st[2] > arena.numel():
        arena = None   # the next backward gets an arena its demand fits (stream order: the old one is idle)
    if arena is None:
        n = max(_FOLD_ARENA_FLOATS, 0 if st is None else (st[2] + (1 << 20)))
        arena = ws["fold_arena"] = torch.empty(n, device=dev)
    return arena


def encoder_backward(cfg, S: EncoderShapes, P, G, prefix, run: EncoderRun, dfeats, pos_emb, len1, len2, *, seed,
                     salt, ws, on_layer_done=None, before_read=None, arena_set=False):
    """dfeats (n_layers, rows, d): grads wrt every hooked layer output (heads + decoder), summed into
    the residual chain as the backward walks down the stack.  on_layer_done(i) is called once layer
    i's parameter gradients are all issued (bucketed all-reduce overlap, kdfm/ddp.py);
    before_read {j: fn}: fn() runs right before dfeats[j] is first read (a stream join for heads
    gradients produced on another stream).  Weight-gradient folds are deferred (fold_arena) and flushed once per
    layer, before on_layer_done; arena_set: the caller already set the arena on the weight-gradient stream (its
    own queued folds are flushed with the first layer's)."""
    dout, dout2 = dfeats[cfg.n_layers - 1], None
    n = cfg.n_layers
    ring = None
    if n >= 2:   # BatchNorm-backward sums: call k uses ring[k] and zeroes ring[(k + 1) % n] for the next call
        ring = ws.get("bn_red_ring")
        if ring is None:
            ring = ws["bn_red_ring"] = torch.zeros(n, 2 * S.d, device=dfeats.device, dtype=torch.float64)
    arena = fold_arena(ws, dfeats.device)
    if arena is not None and not arena_set:
        WGRAD.run(lambda: K.wgrad_set_fold_arena(arena), arena)
    for i in range(cfg.n_layers - 1, -1, -1):
        L = f"{prefix}layers.{i}."
        k = n - 1 - i
        bn_red = None if ring is None else (ring[k], ring[(k + 1) % n])
        # a partial buffer per layer: its LayerNorm fold runs on the weight-gradient stream (LnGrads.fold);
        # layer i's output gradient is dfeats[i] + the gradient layer i + 1 passed down (summed on load by
        # norm_out's LayerNorm backward)
        dx = layer_backward(cfg, S, P, G, L, i, run.layers[i], dout, pos_emb, len2, seed=seed, salt=salt,
                            ln_buf=torch.empty(6, K.layernorm_bwd_ws(S.rows, S.d), device=dfeats.device),
                            dout2=dout2, bn_red=bn_red)
        run.layers[i] = None
        if arena is not None:   # the layer's weight gradients are final after this (before its all-reduce)
            WGRAD.run(K.wgrad_fold_flush)
        if on_layer_done is not None:
            on_layer_done(i)
        if i > 0:
            if before_read is not None and (i - 1) in before_read:
                before_read[i - 1]()
            dout, dout2 = dfeats[i - 1], dx
    subsampling_backward(cfg, S, P, G, prefix, run.sub, dx, len1, seed=seed, salt=salt, ws=ws)
    run.sub = None
    if arena is not None:
        def _end():
            K.wgrad_fold_flush()
            # demand / fallback counters of this backward (host bookkeeping): fold_arena grows the next arena
            ws["fold_stats"] = K.wgrad_fold_stats()
            K.wgrad_set_fold_arena(None)
        WGRAD.run(_end)
    WGRAD.join()  # weight gradients computed on the side stream are complete before anyone reads G


def layer_images(cfg: Ver5Config, P, prefix, d, *, train, dev):
    """The weight images of every fused-kernel product of an encoder's layers (kernels.WeightImages:
    one buffer, one prep launch per step, looked up by ffn_img / lnproj_img / rowgemm_img)."""
    imgs = K.WeightImages(dev)
    ff = cfg.ff_expansion * d
    for i in range(cfg.n_layers):
        L = f"{prefix}layers.{i}."
        if K.ffn_supported(d, ff):
            for which in ("feed_forward1", "feed_forward2"):
                imgs.add(L + which, K.IMG_FFN, P[L + which + ".linear1.weight"], P[L + which + ".linear2.weight"],
                         flag=0 if train else 1, d=d, ff=ff)
        for kind, W in ((K.LNPROJ_QKV, P[L + "self_attn.qkv.weight"]),
                        (K.LNPROJ_GLU, P[L + "conv.pointwise_conv1.weight"].view(2 * d, d))):
            if K.lnproj_supported(kind, d):
                imgs.add(L + f"lnproj{kind}", K.IMG_LNPROJ, W, kind=kind, flag=0, d=d)
            if train and K.lnproj_supported(kind, d, bwd=True):
                imgs.add(L + f"lnproj{kind}_b", K.IMG_LNPROJ, W, kind=kind, flag=1, d=d)
        if K.rowgemm_supported(d):
            for name, W in (("out", P[L + "self_attn.linear_out.weight"]),
                            ("pw2", P[L + "conv.pointwise_conv2.weight"].view(d, d))):
                imgs.add(L + name, K.IMG_ROWGEMM, W, flag=0, d=d)
                if train:
                    imgs.add(L + name + "_t", K.IMG_ROWGEMM, W, flag=1, d=d)
    return imgs.finalize().register()


def make_workspace(S: EncoderShapes, dev):
    ws = {
        "wout_perm": torch.empty(S.d, S.F2, S.C, device=dev),
        "wout_perm_grad": torch.empty(S.d, S.F2, S.C, device=dev),
        "bout_scaled": torch.empty(S.d, device=dev),
    }
    if len(S.stages) == 3 and S.C == S.d:     # 'striding' x4 kernels
        ws["w2_bf16"] = torch.empty(K.subsample_wprep_elems(S.d), device=dev, dtype=torch.bfloat16)
        ws["w2_tapmajor"] = torch.empty(S.d, 9, S.d, device=dev)
        ws["w2_dgrad"] = torch.empty(K.subsample_dgrad_wprep_elems(S.d), device=dev, dtype=torch.bfloat16)
        ws["w2_tapmajor_grad"] = torch.empty(S.d, 9, S.d, device=dev)
        if S.d <= 128 and (S.F2 * S.C) % 4 == 0:
            ws["wout_t_bf16"] = torch.empty(K.ss_out_wprep_elems(S.d, S.F2 * S.C), device=dev, dtype=torch.bfloat16)
        if K.subsample_fused_supported(S.d):
            ws["ss_fused_w"] = torch.empty(K.subsample_fused_wprep_elems(S.d), device=dev, dtype=torch.bfloat16)
    return ws
