"""ORACLE — CPU restatement of the ver5 flow-matching distillation training step.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module, and only as the checker / CPU baseline; the product path
(kd-via-fm-in-asr_amd/kdfm) never imports it.

What it restates (reference = /root/reference, snapshot 2025-09-19):
  * KD heads — literal re-expression of asr_train_diffm.py:400-497 (TeacherAutoEncoder,
    StudentProjector, NoiseAdapter, SimpleDenoiser, FMLatent), :852-856 (rectified schedule
    derivative) and :1270-1427 (FlowMatchingModule, meta_encoder 'mlp', shape_transform 'linear').
    PINNED: tests/test_oracle_golden.py compares it with vectors produced by the reference's own
    classes (tests/golden/make_golden.py, AST-extracted in the survey container).
  * The step — DistilFlowMatchingCTCModelBPE.forward/_compute_v_losses_one_layer/training_step
    (asr_train_diffm.py:606-643, 645-729 [ver5 697-702], 731-828): CTC + 0.1*KL(T=1) +
    sum_16(recon) + sum_16(fm_post).
  * NeMo modules whose sources are present: AudioToMelSpectrogramPreprocessor
    (NeMo/.../modules/audio_preprocessing.py:214-300), ConformerEncoder orchestration
    (conformer_encoder.py:549-850), ConvASRDecoder (conv_asr.py:445-468), CTCLoss
    (losses/ctc.py:25-82, mean_batch + zero_infinity from ctc_models.py:81-85).
  * NeMo leaf modules whose sources are ABSENT (asr/parts/**):
    FilterbankFeatures, ConvSubsampling, RelPositionalEncoding, ConformerLayer and its
    sub-modules.  Restated from the Appendix A contract; pinned only by the invariants of
    NeMo/tests (seq_len = L // hop, zero constant STFT padding); absolute values are
    "parity unpinned" beyond the build's own fixtures.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from .mel import mel_filterbank


@dataclass
class StepConfig:
    n_layers: int = 16
    d_student: int = 88
    heads_student: int = 2
    d_teacher: int = 176
    heads_teacher: int = 4
    latent: int = 96
    vocab: int = 128            # BPE vocabulary; decoder has vocab + 1 classes (blank = vocab)
    conv_kernel: int = 31
    ff_expansion: int = 4
    sample_rate: int = 16000
    n_fft: int = 512
    win: int = 400
    hop: int = 160
    nfilt: int = 80
    preemph: float = 0.97
    dither: float = 1e-5
    fm_steps: int = 8
    denoiser_steps: int = 9
    time_embed_dim: int = 32
    kd_alpha: float = 0.1
    kd_temperature: float = 1.0
    subsampling_mask: bool = True
    subsampling: str = "striding"       # or "dw_striding" (conformer_encoder.py:371-390)
    subsampling_factor: int = 4
    subsampling_conv_channels: int = -1  # -1: d_model
    causal_downsampling: bool = False
    xscaling: bool = True
    version: int = 5                    # --model_version verN (asr_train_diffm.py:1636-1641)
    kd_loss_type: str = "mse"
    use_diffkd: bool = False            # --use_diffkd: DiffKDModule on every layer pair (:795-800)
    # asr_train.py's encoder-level FM family instead of the latent heads (oracle/encfm.py)
    kd_model: str = "diffm"             # "encfm" (asr_train.py) or "logitkd" (DistilEncDecCTCModelBPE)
    encfm_strategy: str = "batch_mode"
    encfm_fixed: tuple = None           # sampling_steps_per_layer (fixed steps, no router) when given
    encfm_meta: str = "mlp"             # FlowMatchingModule meta_encoder_type (mlp | cnn | swin)
    router_max_steps: int = 8
    router_weight: float = 1.0
    flow_schedule: str = "rectified"
    diffkd_steps: int = 9               # --diffkd_steps (diffkd_cfg["diffusion_steps"], :1830-1836)
    bn_momentum: float = 0.1
    ln_eps: float = 1e-5
    bn_eps: float = 1e-5


# ------------------------------------------------------------------------------------------
# Parameter initialisation (NeMo state-dict key names)
# ------------------------------------------------------------------------------------------

def _lin(g, n_out, n_in, bias=True, scale=None):
    s = scale if scale is not None else 1.0 / math.sqrt(n_in)
    w = (torch.rand(n_out, n_in, generator=g) * 2 - 1) * s
    b = (torch.rand(n_out, generator=g) * 2 - 1) * s if bias else None
    return w, b


def sub_pads(cfg) -> tuple:
    """(left, right) zero padding of every stride-2 3x3 subsampling conv: symmetric 1/1, or
    CausalConv2D's kernel-1 / stride-1 = 2/1 with causal_downsampling."""
    return (2, 1) if cfg.causal_downsampling else (1, 1)


def sub_stage_len(l, cfg):
    """calc_length for one stride-2 k=3 stage: floor((l + pl + pr - 3) / 2 + 1) in floating point."""
    pl, pr = sub_pads(cfg)
    return torch.floor((torch.as_tensor(l).double() + pl + pr - 3) / 2.0 + 1.0).long()


def sub_out_features(cfg) -> int:
    f = torch.tensor(cfg.nfilt)
    for _ in range(int(math.log2(cfg.subsampling_factor))):
        f = sub_stage_len(f, cfg)
    return int(f)


def subsampling_param_shapes(cfg: StepConfig, d: int) -> dict:
    C = d if cfg.subsampling_conv_channels == -1 else cfg.subsampling_conv_channels
    if cfg.subsampling == "striding":
        return {"pre_encode.conv.0.weight": (C, 1, 3, 3), "pre_encode.conv.0.bias": (C,),
                "pre_encode.conv.2.weight": (C, C, 3, 3), "pre_encode.conv.2.bias": (C,),
                "pre_encode.out.weight": (d, C * (cfg.nfilt // 4)), "pre_encode.out.bias": (d,)}
    assert cfg.subsampling == "dw_striding", cfg.subsampling
    shapes = {"pre_encode.conv.0.weight": (C, 1, 3, 3), "pre_encode.conv.0.bias": (C,)}
    for s in range(1, int(math.log2(cfg.subsampling_factor))):
        i = 2 + 3 * (s - 1)            # Sequential: conv, ReLU, [dw, pw, ReLU] x (stages - 1)
        shapes[f"pre_encode.conv.{i}.weight"] = (C, 1, 3, 3)
        shapes[f"pre_encode.conv.{i}.bias"] = (C,)
        shapes[f"pre_encode.conv.{i + 1}.weight"] = (C, C, 1, 1)
        shapes[f"pre_encode.conv.{i + 1}.bias"] = (C,)
    shapes["pre_encode.out.weight"] = (d, C * sub_out_features(cfg))
    shapes["pre_encode.out.bias"] = (d,)
    return shapes


def encoder_param_shapes(cfg: StepConfig, d: int, h: int) -> dict:
    dk = d // h
    shapes = subsampling_param_shapes(cfg, d)
    ff = cfg.ff_expansion * d
    for i in range(cfg.n_layers):
        L = f"layers.{i}."
        for n in ("norm_feed_forward1", "norm_self_att", "norm_conv", "norm_feed_forward2", "norm_out"):
            shapes[L + n + ".weight"] = (d,)
            shapes[L + n + ".bias"] = (d,)
        for f in ("feed_forward1", "feed_forward2"):
            shapes[L + f + ".linear1.weight"] = (ff, d)
            shapes[L + f + ".linear1.bias"] = (ff,)
            shapes[L + f + ".linear2.weight"] = (d, ff)
            shapes[L + f + ".linear2.bias"] = (d,)
        for q in ("linear_q", "linear_k", "linear_v", "linear_out"):
            shapes[L + f"self_attn.{q}.weight"] = (d, d)
            shapes[L + f"self_attn.{q}.bias"] = (d,)
        shapes[L + "self_attn.linear_pos.weight"] = (d, d)
        shapes[L + "self_attn.pos_bias_u"] = (h, dk)
        shapes[L + "self_attn.pos_bias_v"] = (h, dk)
        shapes[L + "conv.pointwise_conv1.weight"] = (2 * d, d, 1)
        shapes[L + "conv.pointwise_conv1.bias"] = (2 * d,)
        shapes[L + "conv.depthwise_conv.weight"] = (d, 1, cfg.conv_kernel)
        shapes[L + "conv.depthwise_conv.bias"] = (d,)
        shapes[L + "conv.batch_norm.weight"] = (d,)
        shapes[L + "conv.batch_norm.bias"] = (d,)
        shapes[L + "conv.pointwise_conv2.weight"] = (d, d, 1)
        shapes[L + "conv.pointwise_conv2.bias"] = (d,)
    return shapes


def init_encoder(cfg: StepConfig, d: int, h: int, seed: int, prefix: str = "encoder.") -> dict:
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shp in encoder_param_shapes(cfg, d, h).items():
        if name.endswith("norm_feed_forward1.weight") or ".norm_" in name and name.endswith(".weight"):
            t = 1.0 + 0.1 * (torch.rand(shp, generator=g) * 2 - 1)
        elif "batch_norm.weight" in name:
            t = 1.0 + 0.1 * (torch.rand(shp, generator=g) * 2 - 1)
        elif "pos_bias" in name:
            t = 0.1 * torch.randn(shp, generator=g)
        else:
            fan_in = int(np.prod(shp[1:])) if len(shp) > 1 else shp[0]
            s = 1.0 / math.sqrt(max(1, fan_in))
            t = (torch.rand(shp, generator=g) * 2 - 1) * s
        out[prefix + name] = t.float()
    n_bn = [k for k in out if k.endswith("batch_norm.weight")]
    for k in n_bn:
        base = k[: -len("weight")]
        dd = out[k].shape[0]
        out[base + "running_mean"] = 0.1 * torch.randn(dd, generator=g)
        out[base + "running_var"] = 1.0 + 0.2 * torch.rand(dd, generator=g)
        out[base + "num_batches_tracked"] = torch.zeros((), dtype=torch.int64)
    return out


def init_decoder(cfg: StepConfig, d: int, seed: int, prefix: str = "decoder.") -> dict:
    g = torch.Generator().manual_seed(seed)
    w, b = _lin(g, cfg.vocab + 1, d)
    return {prefix + "decoder_layers.0.weight": w.unsqueeze(-1), prefix + "decoder_layers.0.bias": b}


def init_heads(cfg: StepConfig, seed: int) -> dict:
    """ver5 head parameters with the reference's module names (asr_train_diffm.py:559-564)."""
    g = torch.Generator().manual_seed(seed)
    L, Ct, Cs, E = cfg.latent, cfg.d_teacher, cfg.d_student, cfg.time_embed_dim
    p = {}

    def conv(name, cout, cin, k):
        w, b = _lin(g, cout, cin * k)
        p[name + ".weight"] = w.view(cout, cin, k)
        p[name + ".bias"] = b

    conv("tae.enc", L, Ct, 1)
    conv("tae.dec", Ct, L, 1)
    conv("sproj.proj", L, Cs, 1)
    conv("adapter.gamma_head.0", L, L, 1)
    conv("adapter.gamma_head.2", 1, L, 1)
    conv("denoiser.net.0", L, L, 3)
    conv("denoiser.net.2", L, L, 3)
    for fm in ("fm_latent.fm.", "fm_latent_2.fm."):
        w, b = _lin(g, E, 1)
        p[fm + "time_embed.weight"], p[fm + "time_embed.bias"] = w, b
        w, b = _lin(g, L, L + E)
        p[fm + "meta_encoder.0.weight"], p[fm + "meta_encoder.0.bias"] = w, b
        w, b = _lin(g, L, L)
        p[fm + "meta_encoder.2.weight"], p[fm + "meta_encoder.2.bias"] = w, b
        w, b = _lin(g, L, L)
        p[fm + "shape_transformation_function.weight"] = w
        p[fm + "shape_transformation_function.bias"] = b
    # DiffKDModule (asr_train_diffm.py:326-394): its own linear autoencoder, projector and denoiser
    conv("diffkd.encoder", L, Ct, 1)
    conv("diffkd.decoder", Ct, L, 1)
    conv("diffkd.proj", L, Cs, 1)
    conv("diffkd.denoiser.0", L, L, 3)
    conv("diffkd.denoiser.2", L, L, 3)
    return p


def frontend_buffers(cfg: StepConfig, prefix: str = "preprocessor.featurizer.") -> dict:
    return {
        prefix + "window": torch.hann_window(cfg.win, periodic=False),
        prefix + "fb": torch.tensor(mel_filterbank(cfg.sample_rate, cfg.n_fft, cfg.nfilt, 0.0,
                                                   cfg.sample_rate / 2)).unsqueeze(0),
    }


def init_all(cfg: StepConfig, teacher_seed=0, student_seed=1, heads_seed=2) -> dict:
    p = {}
    p.update(frontend_buffers(cfg))
    p.update(init_encoder(cfg, cfg.d_student, cfg.heads_student, student_seed))
    p.update(init_decoder(cfg, cfg.d_student, student_seed + 100))
    p.update(init_heads(cfg, heads_seed))
    p.update(frontend_buffers(cfg, "teacher.preprocessor.featurizer."))
    p.update(init_encoder(cfg, cfg.d_teacher, cfg.heads_teacher, teacher_seed, "teacher.encoder."))
    p.update(init_decoder(cfg, cfg.d_teacher, teacher_seed + 100, "teacher.decoder."))
    return p


# ------------------------------------------------------------------------------------------
# Frontend (Appendix A.1; NeMo audio_preprocessing.py:93-103, 214-300)
# ------------------------------------------------------------------------------------------

def preprocess(wav, lengths, window, fb, cfg: StepConfig, dither_noise=None):
    seq_len = torch.div(lengths, cfg.hop, rounding_mode="floor")      # pinned: frames - 1
    x = wav.to(window.dtype)   # float32 (parity) or float64 (accuracy reference)
    if dither_noise is not None:
        x = x + cfg.dither * dither_noise
    timemask = torch.arange(x.shape[1]).unsqueeze(0) < lengths.unsqueeze(1)
    x = torch.cat((x[:, :1], x[:, 1:] - cfg.preemph * x[:, :-1]), dim=1)
    x = x.masked_fill(~timemask, 0.0)
    X = torch.stft(x, n_fft=cfg.n_fft, hop_length=cfg.hop, win_length=cfg.win, window=window, center=True,
                   pad_mode="constant", return_complex=True)
    X = torch.view_as_real(X)
    x = torch.sqrt(X.pow(2).sum(-1))
    x = x.pow(2.0)
    x = torch.matmul(fb.to(x.dtype), x)
    x = torch.log(x + 2 ** -24)
    # normalize_batch(per_feature): mean/std over valid frames, (n-1) denominator, std += 1e-5
    B, _, T = x.shape
    valid = torch.arange(T).unsqueeze(0).expand(B, T) < seq_len.unsqueeze(1)
    num = torch.where(valid.unsqueeze(1), x, 0.0).sum(2)
    den = valid.sum(1)
    mean = num / den.unsqueeze(1)
    std = torch.sqrt(torch.sum(torch.where(valid.unsqueeze(1), x - mean.unsqueeze(2), 0.0) ** 2, 2)
                     / (den.unsqueeze(1) - 1.0))
    std = std.masked_fill(std.isnan(), 0.0) + 1e-5
    x = (x - mean.unsqueeze(2)) / std.unsqueeze(2)
    mask = torch.arange(T).repeat(B, 1) >= seq_len.unsqueeze(1)
    x = x.masked_fill(mask.unsqueeze(1), 0.0)
    return x, seq_len


def specaugment_mask(length, T, nfilt, uniforms, freq_masks=2, freq_width=27, time_masks=5, time_width=0.05):
    """SpecAugment mask, NeMo's vectorized form (SpectrogramAugmentation(use_vectorized_spec_augment=True),
    the default at audio_preprocessing.py:490-520 -> SpecAugment._forward_vectorized / _apply_masks;
    SURVEY.md Appendix A.2), with the torch.rand draws given as `uniforms` (B, 2 (time_masks +
    freq_masks)) = per utterance [time widths | time starts | freq widths | freq starts].  Restated with
    the same torch ops, dtypes and order as NeMo's _apply_masks: time axis first (width = time_width *
    length clamped to T, per-utterance float), then frequency (int width).  Returns (B, T, nfilt) bool,
    True = masked.  Parity unpinned against NeMo itself (its source is absent here); the formula is
    SURVEY A.2's."""
    length = torch.as_tensor(length, dtype=torch.int64)
    u = torch.as_tensor(uniforms, dtype=torch.float32).reshape(length.shape[0], -1)
    B = length.shape[0]
    ut_w, ut_s = u[:, :time_masks], u[:, time_masks:2 * time_masks]
    uf_w, uf_s = u[:, 2 * time_masks:2 * time_masks + freq_masks], u[:, 2 * time_masks + freq_masks:]
    # axis 2 (time): width = clamp(width * length, max=axis_length).unsqueeze(1)
    w_t = torch.clamp(time_width * length, max=T).unsqueeze(1)
    mw = (ut_w * w_t).long()
    ms = (ut_s * (length.unsqueeze(1) - mw)).long()
    idx = torch.arange(T)
    tmask = ((idx >= ms.unsqueeze(-1)) & (idx < (ms + mw).unsqueeze(-1))).any(dim=1)      # (B, T)
    # axis 1 (freq): int width
    fw = (uf_w * freq_width).long()
    fs = (uf_s * (nfilt - fw)).long()
    idf = torch.arange(nfilt)
    fmask = ((idf >= fs.unsqueeze(-1)) & (idf < (fs + fw).unsqueeze(-1))).any(dim=1)      # (B, nfilt)
    return tmask[:, :, None] | fmask[:, None, :]


# ------------------------------------------------------------------------------------------
# Encoder (conformer_encoder.py:549-850 + Appendix A.3-A.8)
# ------------------------------------------------------------------------------------------

def _conv_len(l):
    return torch.floor((l.float() - 1.0) / 2.0 + 1.0).long()


def _time_mask(x, lengths, tdim):
    T = x.shape[tdim]
    m = torch.arange(T).unsqueeze(0) < lengths.unsqueeze(1)   # (B,T)
    shape = [x.shape[0]] + [1] * (x.dim() - 1)
    shape[tdim] = T
    return x * m.view(shape).to(x.dtype)


def subsampling_dw_striding(x_btf, lengths, p, pre, cfg: StepConfig):
    """ConvSubsampling 'dw_striding' (built at conformer_encoder.py:381-390 with subsampling
    'dw_striding', recipe fast-conformer_ctc_bpe.yaml:122-125; module source absent, restated):
    Conv2d(1->C, 3, s2) -> ReLU, then (log2(factor) - 1) x [depthwise Conv2d(C, 3, s2, groups=C) ->
    pointwise Conv2d(C->C, 1) -> ReLU], then Linear(C*F' -> d) on (B, T', C*F') (c-major flattening).
    Padding 1/1, or 2/1 (CausalConv2D) with causal_downsampling.  Frames at or past each layer's
    valid length are zeroed before every layer and at the end (the masked conv sequence pinned by
    NeMo/tests/collections/asr/test_padding_and_batch_size_invariance.py:49-130)."""
    pl, pr = sub_pads(cfg)
    mask = cfg.subsampling_mask

    def m(x, L):
        return _time_mask(x, L, 2) if mask else x

    def conv3(x, w, b, groups):
        return F.conv2d(F.pad(x, (pl, pr, pl, pr)), w, b, stride=2, groups=groups)

    x = x_btf.unsqueeze(1)                         # (B,1,T,F)
    L = lengths
    x = conv3(m(x, L), p[pre + "conv.0.weight"], p[pre + "conv.0.bias"], 1)
    L = sub_stage_len(L, cfg)
    x = F.relu(m(x, L))
    C = x.shape[1]
    for s in range(1, int(math.log2(cfg.subsampling_factor))):
        i = 2 + 3 * (s - 1)
        x = conv3(m(x, L), p[pre + f"conv.{i}.weight"], p[pre + f"conv.{i}.bias"], C)
        L = sub_stage_len(L, cfg)
        x = F.conv2d(m(x, L), p[pre + f"conv.{i + 1}.weight"], p[pre + f"conv.{i + 1}.bias"])
        x = F.relu(m(x, L))
    x = m(x, L)
    b, c, t, f = x.shape
    x = x.transpose(1, 2).reshape(b, t, c * f)
    x = F.linear(x, p[pre + "out.weight"], p[pre + "out.bias"])
    return x, L


def subsampling(x_btf, lengths, p, pre, cfg: StepConfig):
    """ConvSubsampling 'striding' factor 4 (A.3); 'dw_striding' dispatches to the function above."""
    if cfg.subsampling == "dw_striding":
        return subsampling_dw_striding(x_btf, lengths, p, pre, cfg)
    x = x_btf.unsqueeze(1)                         # (B,1,T,F)
    l1 = _conv_len(lengths)
    l2 = _conv_len(l1)
    if cfg.subsampling_mask:
        x = _time_mask(x, lengths, 2)
    x = F.relu(F.conv2d(x, p[pre + "conv.0.weight"], p[pre + "conv.0.bias"], stride=2, padding=1))
    if cfg.subsampling_mask:
        x = _time_mask(x, l1, 2)
    x = F.relu(F.conv2d(x, p[pre + "conv.2.weight"], p[pre + "conv.2.bias"], stride=2, padding=1))
    if cfg.subsampling_mask:
        x = _time_mask(x, l2, 2)
    b, c, t, f = x.shape
    x = x.transpose(1, 2).reshape(b, t, c * f)
    x = F.linear(x, p[pre + "out.weight"], p[pre + "out.bias"])
    return x, l2


def rel_pos_emb(T, d, dtype=torch.float32):
    """RelPositionalEncoding (A.4): sinusoids for relative positions T-1 ... -(T-1)."""
    pos = torch.arange(T - 1, -T, -1, dtype=dtype).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=dtype) * -(math.log(10000.0) / d))
    pe = torch.zeros(pos.shape[0], d, dtype=dtype)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.unsqueeze(0)


def rel_shift(x):
    """NeMo RelPositionMultiHeadAttention.rel_shift (A.7), literal pad/view form."""
    b, h, qlen, pos_len = x.size()
    x = F.pad(x, pad=(1, 0))
    x = x.view(b, h, -1, qlen)
    x = x[:, :, 1:].view(b, h, qlen, pos_len)
    return x


def rel_mha(x, pos_emb, att_mask, p, L, h):
    B, T, d = x.shape
    dk = d // h
    q = F.linear(x, p[L + "linear_q.weight"], p[L + "linear_q.bias"]).view(B, T, h, dk)
    k = F.linear(x, p[L + "linear_k.weight"], p[L + "linear_k.bias"]).view(B, T, h, dk).transpose(1, 2)
    v = F.linear(x, p[L + "linear_v.weight"], p[L + "linear_v.bias"]).view(B, T, h, dk).transpose(1, 2)
    pp = F.linear(pos_emb, p[L + "linear_pos.weight"]).view(1, -1, h, dk).transpose(1, 2)
    qu = (q + p[L + "pos_bias_u"]).transpose(1, 2)
    qv = (q + p[L + "pos_bias_v"]).transpose(1, 2)
    bd = rel_shift(torch.matmul(qv, pp.transpose(-2, -1)))
    ac = torch.matmul(qu, k.transpose(-2, -1))
    bd = bd[:, :, :, : ac.size(-1)]
    scores = (ac + bd) / math.sqrt(dk)
    m = att_mask.unsqueeze(1)
    scores = scores.masked_fill(m, -10000.0)
    attn = torch.softmax(scores, dim=-1).masked_fill(m, 0.0)
    o = torch.matmul(attn, v).transpose(1, 2).reshape(B, T, d)
    return F.linear(o, p[L + "linear_out.weight"], p[L + "linear_out.bias"])


def ffn(x, p, L):
    h = F.silu(F.linear(x, p[L + "linear1.weight"], p[L + "linear1.bias"]))
    return F.linear(h, p[L + "linear2.weight"], p[L + "linear2.bias"])


def conv_module(x, pad_mask, p, L, training, bn_state, cfg: StepConfig):
    x = x.transpose(1, 2)
    x = F.conv1d(x, p[L + "pointwise_conv1.weight"], p[L + "pointwise_conv1.bias"])
    x = F.glu(x, dim=1)
    x = x.masked_fill(pad_mask.unsqueeze(1), 0.0)
    d = x.shape[1]
    x = F.conv1d(x, p[L + "depthwise_conv.weight"], p[L + "depthwise_conv.bias"],
                 padding=(cfg.conv_kernel - 1) // 2, groups=d)
    rm, rv = bn_state[L + "batch_norm.running_mean"], bn_state[L + "batch_norm.running_var"]
    x = F.batch_norm(x, rm, rv, p[L + "batch_norm.weight"], p[L + "batch_norm.bias"], training=training,
                     momentum=cfg.bn_momentum, eps=cfg.bn_eps)
    x = F.silu(x)
    x = F.conv1d(x, p[L + "pointwise_conv2.weight"], p[L + "pointwise_conv2.bias"])
    return x.transpose(1, 2)


def conformer_layer(x, pos_emb, att_mask, pad_mask, p, L, h, training, bn_state, cfg: StepConfig):
    def ln(t, n):
        return F.layer_norm(t, (t.shape[-1],), p[L + n + ".weight"], p[L + n + ".bias"], cfg.ln_eps)

    r = x + 0.5 * ffn(ln(x, "norm_feed_forward1"), p, L + "feed_forward1.")
    r = r + rel_mha(ln(r, "norm_self_att"), pos_emb, att_mask, p, L + "self_attn.", h)
    r = r + conv_module(ln(r, "norm_conv"), pad_mask, p, L + "conv.", training, bn_state, cfg)
    r = r + 0.5 * ffn(ln(r, "norm_feed_forward2"), p, L + "feed_forward2.")
    return ln(r, "norm_out")


def encoder(mel, lengths, p, prefix, d, h, cfg: StepConfig, training, bn_state):
    """ConformerEncoder.forward -> (B,d,T') , lengths, [per-layer outputs (B,T',d)]"""
    x = mel.transpose(1, 2)
    x, length = subsampling(x, lengths, p, prefix + "pre_encode.", cfg)
    B, T, _ = x.shape
    if cfg.xscaling:
        x = x * math.sqrt(d)
    pos_emb = rel_pos_emb(T, d, x.dtype)
    valid = torch.arange(T).expand(B, T) < length.unsqueeze(1)
    att_ok = valid.unsqueeze(1).repeat(1, T, 1)
    att_ok = att_ok & att_ok.transpose(1, 2)
    att_mask = ~att_ok
    pad_mask = ~valid
    feats = []
    for i in range(cfg.n_layers):
        x = conformer_layer(x, pos_emb, att_mask, pad_mask, p, prefix + f"layers.{i}.", h, training, bn_state, cfg)
        feats.append(x)
    return x.transpose(1, 2), length, feats


def decoder(enc_bdt, p, prefix):
    logits = F.conv1d(enc_bdt, p[prefix + "decoder_layers.0.weight"], p[prefix + "decoder_layers.0.bias"])
    return F.log_softmax(logits.transpose(1, 2), dim=-1)


def ctc_loss_mean_batch(log_probs, targets, input_lengths, target_lengths, blank):
    loss = F.ctc_loss(log_probs.transpose(0, 1), targets.long(), input_lengths.long(), target_lengths.long(),
                      blank=blank, reduction="none", zero_infinity=True)
    return loss.mean()


# ------------------------------------------------------------------------------------------
# KD heads (asr_train_diffm.py:400-497, 852-856, 1270-1427) — layout (B,C,T) as the reference
# ------------------------------------------------------------------------------------------

def _c1(x, p, name, padding=0):
    return F.conv1d(x, p[name + ".weight"], p[name + ".bias"], padding=padding)


def tae(t_bct, p):
    z = _c1(t_bct, p, "tae.enc")
    return z, _c1(z, p, "tae.dec")


def sproj(s_bct, p):
    return _c1(s_bct, p, "sproj.proj")


def noise_adapter(z, p, eps):
    g = torch.sigmoid(_c1(F.relu(_c1(z, p, "adapter.gamma_head.0")), p, "adapter.gamma_head.2"))
    return g * z + (1.0 - g) * eps, g


def denoiser(z, p, steps):
    x = z
    for _ in range(steps):
        pred = _c1(F.relu(_c1(x, p, "denoiser.net.0", 1)), p, "denoiser.net.2", 1)
        x = x - pred / steps
    return x


def diffkd(s_btd, t_btd, p, steps):
    """DiffKDModule.forward (asr_train_diffm.py:364-394): teacher latent z = encoder(t) DETACHED (the
    encoder never receives a gradient), recon MSE(decoder(z), t), student latent proj(s) denoised by
    `steps` Euler steps x -= denoiser(x) / steps, distill MSE(denoised, z); returns their sum."""
    s = s_btd.permute(0, 2, 1)
    t = t_btd.permute(0, 2, 1)
    z_t = _c1(t, p, "diffkd.encoder").detach()
    ae = F.mse_loss(_c1(z_t, p, "diffkd.decoder"), t)
    x = _c1(s, p, "diffkd.proj")
    for _ in range(steps):
        x = x - _c1(F.relu(_c1(x, p, "diffkd.denoiser.0", 1)), p, "diffkd.denoiser.2", 1) / steps
    return ae + F.mse_loss(x, z_t)


def fm_latent(s_bct, t_bct, p, steps, prefix="fm_latent.fm."):
    """FMLatent.forward -> FlowMatchingModule.forward (training, rectified, mlp, linear)."""
    s_f = s_bct.transpose(1, 2)
    t_f = t_bct.transpose(1, 2)
    x = s_f
    velocity = None
    t = None
    for i in range(steps, 0, -1):
        t = torch.full((s_f.size(0), s_f.size(1), 1), i / steps, dtype=s_f.dtype)
        e = F.linear(t, p[prefix + "time_embed.weight"], p[prefix + "time_embed.bias"])
        h = F.relu(F.linear(torch.cat([x, e], dim=-1), p[prefix + "meta_encoder.0.weight"],
                            p[prefix + "meta_encoder.0.bias"]))
        velocity = F.linear(h, p[prefix + "meta_encoder.2.weight"], p[prefix + "meta_encoder.2.bias"])
        x = x - velocity / steps
    dalpha, dsigma = torch.ones_like(t), -torch.ones_like(t)        # rectified_flow_schedule_deriv
    nsx = (dalpha * s_f - velocity) / (-dsigma)
    tr = F.linear(nsx, p[prefix + "shape_transformation_function.weight"],
                  p[prefix + "shape_transformation_function.bias"])
    return F.mse_loss(tr, t_f), x.transpose(1, 2)


def ver5_layer_losses(s_btd, t_btd, p, eps, cfg: StepConfig):
    """_compute_v_losses_one_layer, version 5 (asr_train_diffm.py:645-702)."""
    s = s_btd.transpose(1, 2)
    t = t_btd.transpose(1, 2)
    z_t, rec = tae(t, p)
    z_t = z_t.detach()
    recon = F.mse_loss(rec, t)
    z_s = sproj(s, p)
    z_noisy, _ = noise_adapter(z_s, p, eps)
    z_deno = denoiser(z_noisy, p, cfg.denoiser_steps)
    fm, _ = fm_latent(z_deno, z_t, p, cfg.fm_steps)
    return recon, fm


def v_layer_losses(version, s_btd, t_btd, p, eps, denoiser_steps=9, fm_steps=8, kd="mse"):
    """_compute_v_losses_one_layer for every version 1-8 (asr_train_diffm.py:645-729); kd_crit is
    nn.MSELoss or nn.L1Loss (:557).  eps: the NoiseAdapter draw (B, L, T) (one adapter call per
    version).  Returns the dict of the five per-layer terms (zeros where the version has none)."""
    s = s_btd.transpose(1, 2)
    t = t_btd.transpose(1, 2)
    z_t, rec = tae(t, p)
    z_t = z_t.detach()
    kd_crit = F.l1_loss if kd == "l1" else F.mse_loss
    zero = torch.zeros(())
    out = {"recon_loss": F.mse_loss(rec, t), "kd_loss_pre": zero, "fm_loss_pre": zero, "kd_loss_post": zero,
           "fm_loss_post": zero}
    z_s = sproj(s, p)

    def deno(z):
        return denoiser(noise_adapter(z, p, eps)[0], p, denoiser_steps)

    def fm(a, prefix="fm_latent.fm."):
        return fm_latent(a, z_t, p, fm_steps, prefix)

    if version == 1:
        out["kd_loss_pre"] = kd_crit(z_s, z_t)
    elif version == 2:
        out["fm_loss_pre"] = fm(z_s)[0]
    elif version == 3:
        out["kd_loss_post"] = kd_crit(deno(z_s), z_t)
    elif version == 4:
        out["fm_loss_pre"] = fm(z_s)[0]
        out["kd_loss_post"] = kd_crit(deno(z_s), z_t)
    elif version == 5:
        out["fm_loss_post"] = fm(deno(z_s))[0]
    elif version == 6:
        out["fm_loss_pre"], x = fm(z_s)
        out["fm_loss_post"] = fm(deno(x), "fm_latent_2.fm.")[0]
    elif version == 7:
        out["fm_loss_pre"] = fm(z_s)[0]
        out["fm_loss_post"] = fm(deno(z_s), "fm_latent_2.fm.")[0]
    elif version == 8:
        out["fm_loss_pre"], x = fm(z_s)
        out["kd_loss_post"] = kd_crit(deno(x), z_t)
    else:
        raise ValueError(version)
    return out


# ------------------------------------------------------------------------------------------
# The whole step
# ------------------------------------------------------------------------------------------

def ver5_step(p, wav, wav_len, targets, target_len, cfg: StepConfig, eps, spec_mask=None,
              student_train=True, bn_state=None, gumbel=None):
    """Forward of one ver5 training step; returns dict of losses and intermediates.

    eps: (n_layers, B, latent, T') NoiseAdapter noise (injected; the reference draws randn_like).
    spec_mask: optional (B, nfilt, T_mel) bool SpecAugment mask (True = masked to 0).
    bn_state: dict of running stats (cloned, updated in place for the student).
    gumbel: kd_model "encfm": per-layer (B, router_max_steps) router Gumbel noise (injected).
    """
    if bn_state is None:
        bn_state = {k: v.clone() for k, v in p.items() if "running_" in k}
    mel, mel_len = preprocess(wav, wav_len, p["preprocessor.featurizer.window"],
                              p["preprocessor.featurizer.fb"][0], cfg)
    mel_s = mel.masked_fill(spec_mask, 0.0) if spec_mask is not None else mel
    enc, enc_len, s_feats = encoder(mel_s, mel_len, p, "encoder.", cfg.d_student, cfg.heads_student, cfg,
                                    student_train, bn_state)
    with torch.no_grad():
        mel_t, mel_t_len = preprocess(wav, wav_len, p["teacher.preprocessor.featurizer.window"],
                                      p["teacher.preprocessor.featurizer.fb"][0], cfg)
        _, _, t_feats = encoder(mel_t, mel_t_len, p, "teacher.encoder.", cfg.d_teacher, cfg.heads_teacher, cfg,
                                False, bn_state)
    encfm_out = None
    if cfg.kd_model == "encfm":
        # asr_train.py:595-666: router + FM over the hooked layer pairs; the decoder reads the last
        # layer's FM output (hook layout (B, T, C) -> the decoder's (B, C, T))
        from oracle import encfm as E
        if cfg.encfm_fixed is not None:
            encfm_out = E.encfm_fixed_forward(p, s_feats, t_feats, cfg.encfm_fixed, schedule=cfg.flow_schedule,
                                              meta=cfg.encfm_meta, heads=cfg.heads_student)
        else:
            encfm_out = E.encfm_forward(p, s_feats, t_feats, gumbel, strategy=cfg.encfm_strategy,
                                        max_steps=cfg.router_max_steps, router_weight=cfg.router_weight,
                                        schedule=cfg.flow_schedule)
        enc = encfm_out["fm_out"].transpose(1, 2)
    log_probs = decoder(enc, p, "decoder.")
    ctc = ctc_loss_mean_batch(log_probs, targets, enc_len, target_len, cfg.vocab)
    with torch.no_grad():
        tch_logp = decoder(t_feats[-1].permute(0, 2, 1), p, "teacher.decoder.")
        tch_p = F.softmax(tch_logp / cfg.kd_temperature, dim=-1)
    stu_logp = F.log_softmax(log_probs / cfg.kd_temperature, dim=-1)
    kl = F.kl_div(stu_logp, tch_p, reduction="batchmean") * cfg.kd_temperature ** 2
    if cfg.kd_model == "logitkd":
        # DistilEncDecCTCModelBPE.training_step (asr_train_diffm.py:243-321): ctc + kd_alpha * logit KD; the
        # KL is the same as ver5's (log_softmax(s/T) vs softmax(teacher log-probs / T), batchmean, * T^2)
        zero = torch.zeros((), dtype=log_probs.dtype)
        return {"loss": ctc + cfg.kd_alpha * kl, "ctc": ctc, "kl": kl, "recon": zero, "fm": zero, "diffkd": zero,
                "log_probs": log_probs, "enc_len": enc_len, "mel": mel, "mel_len": mel_len, "s_feats": s_feats,
                "t_feats": t_feats, "bn_state": bn_state}
    if encfm_out is not None:
        # training_step (asr_train.py:762-768): ctc + kd_alpha * logit_kd + forward's total_loss
        zero = torch.zeros((), dtype=log_probs.dtype)
        total = ctc + cfg.kd_alpha * kl + encfm_out["total"]
        return {"loss": total, "ctc": ctc, "kl": kl, "recon": zero, "fm": encfm_out["total"], "diffkd": zero,
                "encfm": encfm_out, "log_probs": log_probs, "enc_len": enc_len, "mel": mel, "mel_len": mel_len,
                "s_feats": s_feats, "t_feats": t_feats, "bn_state": bn_state}
    recon_sum = torch.zeros((), dtype=log_probs.dtype)
    fm_sum = torch.zeros((), dtype=log_probs.dtype)     # ver5: fm_post; other versions: all four KD terms
    terms = {k: torch.zeros((), dtype=log_probs.dtype) for k in ("kd_loss_pre", "fm_loss_pre", "kd_loss_post",
                                                                 "fm_loss_post")}
    for i, (s, t) in enumerate(zip(s_feats, t_feats)):
        if cfg.version == 5:
            r, f = ver5_layer_losses(s, t, p, eps[i], cfg)
            terms["fm_loss_post"] = terms["fm_loss_post"] + f
        else:
            o = v_layer_losses(cfg.version, s, t, p, eps[i], cfg.denoiser_steps, cfg.fm_steps, cfg.kd_loss_type)
            r = o["recon_loss"]
            f = o["kd_loss_pre"] + o["fm_loss_pre"] + o["kd_loss_post"] + o["fm_loss_post"]
            for k in terms:
                terms[k] = terms[k] + o[k]
        recon_sum = recon_sum + r
        fm_sum = fm_sum + f
    # (optional) DiffKD: mean over the layer pairs (asr_train_diffm.py:795-800)
    dkd = torch.zeros((), dtype=log_probs.dtype)
    if cfg.use_diffkd:
        for s, t in zip(s_feats, t_feats):
            dkd = dkd + diffkd(s, t, p, cfg.diffkd_steps)
        dkd = dkd / max(1, len(s_feats))
    # training_step (asr_train_diffm.py:803-811): ctc + kd_alpha * logit_kd + recon + kd/fm pre/post + diffkd
    total = ctc + cfg.kd_alpha * kl + recon_sum + fm_sum + dkd
    return {"loss": total, "ctc": ctc, "kl": kl, "recon": recon_sum, "fm": fm_sum + dkd, "diffkd": dkd,
            "terms": terms,
            "log_probs": log_probs,
            "enc_len": enc_len, "mel": mel, "mel_len": mel_len, "s_feats": s_feats, "t_feats": t_feats,
            "bn_state": bn_state}


def trainable_names(p: dict, version: int = 5, use_diffkd: bool = False, kd_model: str = "diffm") -> list:
    """Names of the parameters the step trains (teacher frozen; buffers/running stats excluded;
    fm_latent_2 is used by versions 6 and 7 only, and otherwise receives no gradient; the DiffKD
    module only with use_diffkd, and its encoder never: its output is detached before every use)."""
    out = []
    for k, v in p.items():
        if k.startswith("teacher.") or k.startswith("preprocessor.") or "running_" in k or "num_batches" in k:
            continue
        if k.startswith("fm_latent_2.") and version not in (6, 7):
            continue
        if k.startswith("diffkd.") and (not use_diffkd or k.startswith("diffkd.encoder.")):
            continue
        if k.startswith("layer_proj."):   # built with flow matching, used only by layerwise KD (asr_train.py:525-529)
            continue
        if kd_model == "logitkd" and not k.startswith(("encoder.", "decoder.")):
            continue
        out.append(k)
    return out


def greedy_ctc(log_probs, lengths, blank):
    """CTC greedy decode ids (A.9): argmax, collapse repeats, drop blank."""
    out = []
    am = log_probs.argmax(-1)
    for b in range(am.shape[0]):
        prev = -1
        seq = []
        for t in range(int(lengths[b])):
            c = int(am[b, t])
            if c != prev and c != blank:
                seq.append(c)
            prev = c
        out.append(seq)
    return out
