"""Configuration and NeMo state-dict naming of the ver5 FM-distillation step.

Defaults follow the reference's canonical run (scripts/train/diffm_libri100_ver5.sh:10-26 ->
asr_train_diffm.py argparse :1430-1648, ver5 construction :1892-1900) on the Conformer-CTC-small
teacher recipe (NeMo/examples/asr/conf/conformer/conformer_ctc_bpe.yaml:10, 93-157, 180-196) with
the student halved (asr_train_diffm.py:128-130).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace


@dataclass
class Ver5Config:
    # model
    n_layers: int = 16
    d_student: int = 88
    heads_student: int = 2
    d_teacher: int = 176
    heads_teacher: int = 4
    latent: int = 96
    vocab: int = 128                 # decoder emits vocab + 1 classes, blank = vocab
    conv_kernel: int = 31
    ff_expansion: int = 4
    # frontend (FilterbankFeatures defaults, audio_preprocessing.py:216-243)
    sample_rate: int = 16000
    n_fft: int = 512
    win: int = 400
    hop: int = 160
    nfilt: int = 80
    preemph: float = 0.97
    dither: float = 1e-5
    log_guard: float = 2.0 ** -24
    # SpecAugment (conformer_ctc_bpe.yaml:108-114, Small row of the table at :10 -> 5 time masks)
    specaug: bool = True
    freq_masks: int = 2
    freq_width: int = 27
    time_masks: int = 5
    time_width: float = 0.05
    # heads (asr_train_diffm.py:539, 1804-1837); version = --model_version verN (:1636-1641, 645-729),
    # kd_loss_type = the kd_crit of versions 1/3/4/8 (:527, 556)
    version: int = 5
    kd_loss_type: str = "mse"
    fm_steps: int = 8
    denoiser_steps: int = 9
    # --use_diffkd / --diffkd_steps: the DiffKD module on every layer pair, mean over the layers
    # (asr_train_diffm.py:326-394, :795-800), on top of the version's heads
    use_diffkd: bool = False
    diffkd_steps: int = 9
    time_embed_dim: int = 32
    # model family: "diffm" = asr_train_diffm.py's latent KD heads (model versions 1-8 above);
    # "encfm" = asr_train.py's encoder-level flow matching on every hooked layer pair with the
    # DynamicStepRouter (use_flow_matching, :469-666, 1021-1377): per-layer step counts from the router
    # (encfm_dynamic, the --use_dynamic_steps path) turned into FM calls by encfm_strategy
    # (--router_strategy), or fixed per layer (encfm_steps_per_layer = --sampling_steps_per_layer);
    # router_max_steps = --router_max_sampling_steps, router_weight = --router_weight,
    # flow_schedule = --flow_schedule (rectified | vp_ode); "logitkd" = the baseline DistilEncDecCTCModelBPE
    # (CTC + kd_alpha * logit KD only, asr_train_diffm.py:170-324)
    kd_model: str = "diffm"
    encfm_strategy: str = "batch_mode"
    encfm_dynamic: bool = True
    encfm_steps_per_layer: tuple = None
    # --flow_steps (flow_cfg training_sampling): the per-layer count of the fixed-step path when
    # encfm_steps_per_layer is None.  The reference reads it from self.flow_cfg, which its __init__
    # never sets (asr_train.py:644 vs :498-529: AttributeError -- every flowkd_* launcher without
    # --sampling_steps_per_layer stops there); the engine runs the value that line names.
    encfm_flow_steps: int = 8
    # FlowMatchingModule meta_encoder_type (--meta_encoder_type, asr_train.py:1241-1279): "mlp" (router or
    # fixed steps, kdfm/encfm.py) or "cnn" / "swin" / "conformer" / "unet" (fixed steps, kdfm/fmmeta.py;
    # "unet" runs only at an even frame count, as in the reference)
    encfm_meta: str = "mlp"
    # flow_cfg hidden_dim (--hidden_dim, asr_train.py:1753): the U-Net meta-encoder's base width (UNet1D
    # base_ch, :1271-1276); the mlp meta-encoder and the router are built for 128 (ENCFM_HIDDEN)
    encfm_hidden: int = 128
    router_max_steps: int = 8
    router_weight: float = 1.0
    flow_schedule: str = "rectified"
    kd_alpha: float = 0.1
    kd_temperature: float = 1.0
    # regularisation (conformer_ctc_bpe.yaml:150-153)
    dropout: float = 0.1
    dropout_pre: float = 0.1
    dropout_att: float = 0.1
    subsampling_mask: bool = True
    # ConvSubsampling (conformer_encoder.py:371-390): "striding" (Conformer-CTC recipe, x4) or
    # "dw_striding" (FastConformer recipe fast-conformer_ctc_bpe.yaml:122-125: x8, 256 channels)
    subsampling: str = "striding"
    subsampling_factor: int = 4
    subsampling_conv_channels: int = -1   # -1: d_model
    causal_downsampling: bool = False
    xscaling: bool = True                 # x * sqrt(d_model) after subsampling (RelPositionalEncoding)
    bn_momentum: float = 0.1
    ln_eps: float = 1e-5
    bn_eps: float = 1e-5
    # optimizer (teacher .nemo optim: adamw + NoamAnnealing; Small lr 5.0)
    lr: float = 5.0
    betas: tuple = (0.9, 0.98)
    weight_decay: float = 1e-3
    adam_eps: float = 1e-8
    warmup_steps: int = 10000
    min_lr: float = 1e-6
    sched_d_model: int = 88
    # execution
    math: str = "bf16"               # MFMA arithmetic: "bf16" (throughput) or "f32" (parity)
    deterministic: bool = False      # ordered reductions (kdfm_set_deterministic): bitwise-reproducible runs
    # fp8 e4m3 operands (MX: an e8m0 scale per 32 contraction elements, block-scaled MFMA) for the wide Linear products' forward and data
    # gradients on the large-tile route (d_model >= 512: BASELINE.json configs[4] "fp8 MFMA attention/FFN" -- the
    # attention projections and the FFN; the attention core and the weight gradients stay bf16)
    linear_fp8: bool = False
    # opt-in gradient check (not in the reference): global gradient norm + non-finite count each step
    # (kdfm_grad_stats, logged as grad_norm / grad_nonfinite); a non-finite gradient skips the AdamW update
    grad_check: bool = False
    share_frontend: bool = True      # one mel frontend for student+teacher when dither == 0

    @property
    def classes(self) -> int:
        return self.vocab + 1

    def parity(self) -> "Ver5Config":
        """Deterministic fp32 configuration used against the oracle."""
        return replace(self, dither=0.0, specaug=False, dropout=0.0, dropout_pre=0.0, dropout_att=0.0, math="f32",
                       deterministic=True)


# ------------------------------------------------------------------------------------------------
# NeMo state-dict names.  The order below is also the layout of the flat
# parameter buffer: q/k/v weights (and biases) are adjacent so one (3d, d) GEMM projects all three.
# ------------------------------------------------------------------------------------------------

def sub_stages(cfg: Ver5Config) -> int:
    """Number of stride-2 stages of the subsampling module (log2 of the factor)."""
    f = cfg.subsampling_factor
    if f < 2 or f & (f - 1):
        raise ValueError("subsampling_factor must be a power of 2")
    if cfg.subsampling == "striding":
        if f != 4 or cfg.causal_downsampling:
            raise ValueError("'striding' subsampling is implemented for the Conformer-CTC recipe (x4, non-causal)")
    elif cfg.subsampling != "dw_striding":
        raise ValueError(f"subsampling {cfg.subsampling!r} is not on this path (striding | dw_striding)")
    return f.bit_length() - 1


def sub_pad(cfg: Ver5Config) -> tuple:
    """(left, right) padding of every 3x3 stride-2 subsampling conv: 1/1, or CausalConv2D's 2/1."""
    return (2, 1) if cfg.causal_downsampling else (1, 1)


def sub_channels(cfg: Ver5Config, d: int) -> int:
    return d if cfg.subsampling_conv_channels == -1 else cfg.subsampling_conv_channels


def sub_len(cfg: Ver5Config, n: int) -> int:
    """NeMo calc_length for one stage (host ints): floor((n + pl + pr - 3) / 2) + 1."""
    pl, pr = sub_pad(cfg)
    return (n + pl + pr - 3) // 2 + 1


def sub_dims(cfg: Ver5Config, T_mel: int) -> list:
    """[(T, F)] of the input and of every stage output."""
    out = [(T_mel, cfg.nfilt)]
    for _ in range(sub_stages(cfg)):
        t, f = out[-1]
        out.append((sub_len(cfg, t), sub_len(cfg, f)))
    return out


def subsampling_specs(cfg: Ver5Config, d: int, prefix: str) -> list:
    C = sub_channels(cfg, d)
    n = sub_stages(cfg)
    Fo = sub_dims(cfg, 1)[-1][1]
    p = prefix + "pre_encode."
    if cfg.subsampling == "striding":
        return [(p + "conv.0.weight", (C, 1, 3, 3)), (p + "conv.0.bias", (C,)),
                (p + "conv.2.weight", (C, C, 3, 3)), (p + "conv.2.bias", (C,)),
                (p + "out.weight", (d, C * Fo)), (p + "out.bias", (d,))]
    s = [(p + "conv.0.weight", (C, 1, 3, 3)), (p + "conv.0.bias", (C,))]
    for st in range(1, n):
        i = 2 + 3 * (st - 1)     # nn.Sequential: conv, ReLU, [dw, pw, ReLU] x (stages - 1)
        s += [(p + f"conv.{i}.weight", (C, 1, 3, 3)), (p + f"conv.{i}.bias", (C,)),
              (p + f"conv.{i + 1}.weight", (C, C, 1, 1)), (p + f"conv.{i + 1}.bias", (C,))]
    return s + [(p + "out.weight", (d, C * Fo)), (p + "out.bias", (d,))]


def encoder_specs(cfg: Ver5Config, d: int, h: int, prefix: str) -> list:
    ff = cfg.ff_expansion * d
    dk = d // h
    s = subsampling_specs(cfg, d, prefix)
    for i in range(cfg.n_layers):
        L = f"{prefix}layers.{i}."
        s += [(L + "norm_feed_forward1.weight", (d,)), (L + "norm_feed_forward1.bias", (d,)),
              (L + "feed_forward1.linear1.weight", (ff, d)), (L + "feed_forward1.linear1.bias", (ff,)),
              (L + "feed_forward1.linear2.weight", (d, ff)), (L + "feed_forward1.linear2.bias", (d,)),
              (L + "norm_self_att.weight", (d,)), (L + "norm_self_att.bias", (d,)),
              (L + "self_attn.linear_q.weight", (d, d)), (L + "self_attn.linear_k.weight", (d, d)),
              (L + "self_attn.linear_v.weight", (d, d)),
              (L + "self_attn.linear_q.bias", (d,)), (L + "self_attn.linear_k.bias", (d,)),
              (L + "self_attn.linear_v.bias", (d,)),
              (L + "self_attn.linear_out.weight", (d, d)), (L + "self_attn.linear_out.bias", (d,)),
              (L + "self_attn.linear_pos.weight", (d, d)),
              (L + "self_attn.pos_bias_u", (h, dk)), (L + "self_attn.pos_bias_v", (h, dk)),
              (L + "norm_conv.weight", (d,)), (L + "norm_conv.bias", (d,)),
              (L + "conv.pointwise_conv1.weight", (2 * d, d, 1)), (L + "conv.pointwise_conv1.bias", (2 * d,)),
              (L + "conv.depthwise_conv.weight", (d, 1, cfg.conv_kernel)), (L + "conv.depthwise_conv.bias", (d,)),
              (L + "conv.batch_norm.weight", (d,)), (L + "conv.batch_norm.bias", (d,)),
              (L + "conv.pointwise_conv2.weight", (d, d, 1)), (L + "conv.pointwise_conv2.bias", (d,)),
              (L + "norm_feed_forward2.weight", (d,)), (L + "norm_feed_forward2.bias", (d,)),
              (L + "feed_forward2.linear1.weight", (ff, d)), (L + "feed_forward2.linear1.bias", (ff,)),
              (L + "feed_forward2.linear2.weight", (d, ff)), (L + "feed_forward2.linear2.bias", (d,)),
              (L + "norm_out.weight", (d,)), (L + "norm_out.bias", (d,))]
    return s


def bn_buffer_specs(cfg: Ver5Config, d: int, prefix: str) -> list:
    s = []
    for i in range(cfg.n_layers):
        L = f"{prefix}layers.{i}.conv.batch_norm."
        s += [(L + "running_mean", (d,)), (L + "running_var", (d,))]
    return s


def decoder_specs(cfg: Ver5Config, d: int, prefix: str) -> list:
    return [(prefix + "decoder_layers.0.weight", (cfg.classes, d, 1)), (prefix + "decoder_layers.0.bias", (cfg.classes,))]


def head_modules(cfg: Ver5Config) -> tuple:
    """The KD head modules a model version trains (asr_train_diffm.py:645-729): the rest of the
    reference's heads exist in its state dict but never receive a gradient, so AdamW (which skips
    params whose .grad is None) never touches them — they are kept out of the trained buffer."""
    v = cfg.version
    if v not in range(1, 9):
        raise ValueError(f"model version must be 1..8, got {v}")
    if cfg.kd_loss_type not in ("mse", "l1"):
        raise ValueError("kd_loss_type must be 'mse' or 'l1'")
    mods = ["tae", "sproj"]
    if v >= 3:
        mods += ["adapter", "denoiser"]
    if v in (2, 4, 5, 6, 7, 8):
        mods.append("fm_latent")
    if v in (6, 7):
        mods.append("fm_latent_2")
    return tuple(mods)


ENCFM_HIDDEN = 128     # FlowMatchingModule hidden_dim (asr_train.py:1753); the router's proj / hidden widths
ENCFM_ROUTER_EMB = 32  # DynamicStepRouter layer_emb_dim (:514)


def encfm_fixed_steps(cfg: Ver5Config) -> tuple:
    """Per-layer FM step counts of the fixed-step path (use_dynamic_steps False, asr_train.py:639-645):
    sampling_steps_per_layer when given, else training_sampling (= --flow_steps) for every layer."""
    if cfg.encfm_steps_per_layer is not None:
        steps = tuple(int(s) for s in cfg.encfm_steps_per_layer)
    else:
        steps = (int(cfg.encfm_flow_steps),) * cfg.n_layers
    if len(steps) != cfg.n_layers or not all(1 <= s <= cfg.router_max_steps for s in steps):
        raise ValueError(f"fixed FM step counts {steps}: need one count in [1, router_max_steps="
                         f"{cfg.router_max_steps}] per layer ({cfg.n_layers})")
    return steps


def meta_specs(cfg: Ver5Config) -> list:
    """FlowMatchingModule.meta_encoder parameters for cfg.encfm_meta (asr_train.py:1244-1259, 844-851)."""
    Cs, E, H = cfg.d_student, cfg.time_embed_dim, ENCFM_HIDDEN
    Ci = Cs + E
    me = "flow_matching.meta_encoder."
    if cfg.encfm_meta == "mlp":
        return [(me + "0.weight", (H, Ci)), (me + "0.bias", (H,)), (me + "2.weight", (Cs, H)), (me + "2.bias", (Cs,))]
    if cfg.encfm_meta == "cnn":
        return [(me + "0.weight", (Cs, Ci, 3)), (me + "0.bias", (Cs,)), (me + "2.weight", (Cs, Cs, 1)),
                (me + "2.bias", (Cs,))]
    if cfg.encfm_meta == "swin":
        return [(me + "attn.in_proj_weight", (3 * Ci, Ci)), (me + "attn.in_proj_bias", (3 * Ci,)),
                (me + "attn.out_proj.weight", (Ci, Ci)), (me + "attn.out_proj.bias", (Ci,)),
                (me + "linear1.weight", (Cs, Ci)), (me + "linear1.bias", (Cs,)),
                (me + "linear2.weight", (Cs, Cs)), (me + "linear2.bias", (Cs,))]
    if cfg.encfm_meta == "conformer":   # ConformerEncoder (:1000-1020), kdfm/fmconf.py
        from .fmconf import conformer_specs
        return conformer_specs(Cs, E)
    if cfg.encfm_meta == "unet":   # UNet1D(in Ci, base hidden_dim, out Cs, 4 layers) (:880-917, 1271-1276)
        return unet_specs(Cs, E, cfg.encfm_hidden)
    raise ValueError(f"encfm_meta must be 'mlp', 'cnn', 'swin', 'conformer' or 'unet', got {cfg.encfm_meta!r}")


UNET_LAYERS = 4   # UNet1D num_layers (asr_train.py:1275)


def unet_channels(Cs, E, base, layers=UNET_LAYERS):
    """UNet1D's widths: down i maps c_in[i] -> c_down[i] = base 2^i (Conv1d k 4 s 2 p 1); the bottleneck keeps
    c_down[-1]; up j maps c_up_in[j] = c_prev + skip (deepest skip first) -> that skip's width."""
    cin = [Cs + E] + [base * 2 ** i for i in range(layers - 1)]
    cdown = [base * 2 ** i for i in range(layers)]
    ups, ch = [], cdown[-1]
    for skip in reversed(cdown):
        ups.append((ch + skip, skip))
        ch = skip
    return cin, cdown, ups


def unet_specs(Cs, E, base, layers=UNET_LAYERS):
    me = "flow_matching.meta_encoder."
    cin, cdown, ups = unet_channels(Cs, E, base, layers)
    s = []
    for i in range(layers):
        s += [(me + f"downs.{i}.weight", (cdown[i], cin[i], 4)), (me + f"downs.{i}.bias", (cdown[i],))]
    s += [(me + "bottleneck.weight", (cdown[-1], cdown[-1], 3)), (me + "bottleneck.bias", (cdown[-1],))]
    for j, (ci, co) in enumerate(ups):   # ConvTranspose1d weight: (in, out, k)
        s += [(me + f"ups.{j}.weight", (ci, co, 4)), (me + f"ups.{j}.bias", (co,))]
    s += [(me + "final.weight", (Cs, cdown[0], 1)), (me + "final.bias", (Cs,))]
    return s


def meta_bn_specs(cfg: Ver5Config) -> list:
    """BatchNorm running statistics of the FM meta-encoder (the conformer's 4 ConvModules), kept beside the
    encoders' in the engine's buffer store."""
    if cfg.kd_model != "encfm" or cfg.encfm_meta != "conformer":
        return []
    from .fmconf import bn_buffer_specs as conf_bn
    return conf_bn(cfg.d_student)


def encfm_specs(cfg: Ver5Config, trained: bool = True) -> list:
    """Parameters of the encoder-level FM family, named as the reference module tree.  trained:
    flow_matching.* and (dynamic steps) router.*; else the ones the reference builds but never trains:
    layer_proj (built whenever flow matching is on, asr_train.py:525-529, used only by layerwise KD) and
    the router when the step counts are fixed."""
    Cs, Ct, E, H = cfg.d_student, cfg.d_teacher, cfg.time_embed_dim, ENCFM_HIDDEN
    fm = "flow_matching."
    fm_specs = [(fm + "time_embed.weight", (E, 1)), (fm + "time_embed.bias", (E,))] + meta_specs(cfg) + [
                (fm + "shape_transformation_function.weight", (Ct, Cs)),
                (fm + "shape_transformation_function.bias", (Ct,))]
    r = "router."
    router_specs = [(r + "stu_proj.0.weight", (H, Cs)), (r + "stu_proj.0.bias", (H,)),
                    (r + "tch_proj.0.weight", (H, Ct)), (r + "tch_proj.0.bias", (H,)),
                    (r + "layer_emb.weight", (cfg.n_layers, ENCFM_ROUTER_EMB)),
                    (r + "router.0.weight", (H, 2 * H + ENCFM_ROUTER_EMB)), (r + "router.0.bias", (H,)),
                    (r + "router.2.weight", (cfg.router_max_steps, H)), (r + "router.2.bias", (cfg.router_max_steps,))]
    if trained:
        return fm_specs + (router_specs if cfg.encfm_dynamic else [])
    return (router_specs if not cfg.encfm_dynamic else []) + [("layer_proj.weight", (Ct, Cs)),
                                                              ("layer_proj.bias", (Ct,))]


def head_specs(cfg: Ver5Config, fm_prefixes=None) -> list:
    if cfg.kd_model == "encfm":
        if cfg.use_diffkd:
            # asr_train.py runs DiffKD beside the encoder-level FM (latent = the student width, loss summed
            # over the layers, :754-767, 1776-1782); the engine does not: refuse rather than train its
            # parameters on zero gradients
            raise ValueError("kd_model='encfm' with use_diffkd is not supported by the engine")
        if cfg.encfm_meta != "mlp" and cfg.encfm_dynamic:
            raise ValueError(f"encfm_meta={cfg.encfm_meta!r} runs with fixed step counts (encfm_dynamic=False, "
                             "encfm_steps_per_layer); the dynamic router drives the 'mlp' meta-encoder only")
        return encfm_specs(cfg, True)
    if cfg.kd_model == "logitkd":
        # DistilEncDecCTCModelBPE (asr_train_diffm.py:170-324, asr_train.py:314-466; the logitkd_* launchers):
        # CTC + kd_alpha * logit KD, no latent heads.  Its use_layerwise_distillation branch builds a fresh
        # projection lazily after the optimizer exists (never trained) and stays out of scope
        if cfg.use_diffkd:
            raise ValueError("kd_model='logitkd' has no DiffKD module")
        return []
    if cfg.kd_model != "diffm":
        raise ValueError(f"kd_model must be 'diffm', 'encfm' or 'logitkd', got {cfg.kd_model!r}")
    L, Ct, Cs, E = cfg.latent, cfg.d_teacher, cfg.d_student, cfg.time_embed_dim
    mods = head_modules(cfg)
    s = [("tae.enc.weight", (L, Ct, 1)), ("tae.enc.bias", (L,)),
         ("tae.dec.weight", (Ct, L, 1)), ("tae.dec.bias", (Ct,)),
         ("sproj.proj.weight", (L, Cs, 1)), ("sproj.proj.bias", (L,))]
    if "adapter" in mods:
        s += [("adapter.gamma_head.0.weight", (L, L, 1)), ("adapter.gamma_head.0.bias", (L,)),
              ("adapter.gamma_head.2.weight", (1, L, 1)), ("adapter.gamma_head.2.bias", (1,)),
              ("denoiser.net.0.weight", (L, L, 3)), ("denoiser.net.0.bias", (L,)),
              ("denoiser.net.2.weight", (L, L, 3)), ("denoiser.net.2.bias", (L,))]
    if fm_prefixes is None:
        fm_prefixes = [m + ".fm." for m in mods if m.startswith("fm_latent")]
    for fm in fm_prefixes:
        s += [(fm + "time_embed.weight", (E, 1)), (fm + "time_embed.bias", (E,)),
              (fm + "meta_encoder.0.weight", (L, L + E)), (fm + "meta_encoder.0.bias", (L,)),
              (fm + "meta_encoder.2.weight", (L, L)), (fm + "meta_encoder.2.bias", (L,)),
              (fm + "shape_transformation_function.weight", (L, L)),
              (fm + "shape_transformation_function.bias", (L,))]
    return s


def diffkd_specs(cfg: Ver5Config, trained: bool) -> list:
    """DiffKDModule parameters (asr_train_diffm.py:341-358): trained = decoder, proj, denoiser; the
    encoder never receives a gradient (its output is detached before every use, :382-383)."""
    L, Ct, Cs = cfg.latent, cfg.d_teacher, cfg.d_student
    if not trained:
        return [("diffkd.encoder.weight", (L, Ct, 1)), ("diffkd.encoder.bias", (L,))]
    return [("diffkd.decoder.weight", (Ct, L, 1)), ("diffkd.decoder.bias", (Ct,)),
            ("diffkd.proj.weight", (L, Cs, 1)), ("diffkd.proj.bias", (L,)),
            ("diffkd.denoiser.0.weight", (L, L, 3)), ("diffkd.denoiser.0.bias", (L,)),
            ("diffkd.denoiser.2.weight", (L, L, 3)), ("diffkd.denoiser.2.bias", (L,))]


def all_head_specs(cfg: Ver5Config) -> list:
    """Every KD head the reference module builds, whatever the version (asr_train_diffm.py:559-564):
    version 6 uses all of them."""
    from dataclasses import replace
    if cfg.kd_model == "encfm":
        return encfm_specs(cfg, True) + encfm_specs(cfg, False)
    if cfg.kd_model == "logitkd":
        return []
    return head_specs(replace(cfg, version=6))


def student_specs(cfg: Ver5Config) -> list:
    """Trainable parameters of the step: student encoder + decoder + the heads the version uses
    (head_modules; for ver5 fm_latent_2 exists in the reference but never receives a gradient)."""
    return (encoder_specs(cfg, cfg.d_student, cfg.heads_student, "encoder.")
            + decoder_specs(cfg, cfg.d_student, "decoder.") + head_specs(cfg)
            + (diffkd_specs(cfg, True) if cfg.use_diffkd else []))


def teacher_specs(cfg: Ver5Config) -> list:
    return (encoder_specs(cfg, cfg.d_teacher, cfg.heads_teacher, "teacher.encoder.")
            + decoder_specs(cfg, cfg.d_teacher, "teacher.decoder."))


def fused_groups(specs: list) -> dict:
    """name of fused view -> (first member, count, fused shape): q|k|v weights and biases."""
    out = {}
    names = [n for n, _ in specs]
    shapes = dict(specs)
    for n in names:
        if n.endswith("self_attn.linear_q.weight"):
            base = n[: -len("linear_q.weight")]
            d = shapes[n][0]
            out[base + "qkv.weight"] = (n, 3, (3 * d, d))
            out[base + "qkv.bias"] = (base + "linear_q.bias", 3, (3 * d,))
    return out


DEFAULT = Ver5Config()
PARITY = DEFAULT.parity()

__all__ = ["Ver5Config", "DEFAULT", "PARITY", "encoder_specs", "subsampling_specs", "sub_stages", "sub_pad",
           "sub_channels", "sub_len", "sub_dims", "decoder_specs", "head_specs", "all_head_specs", "diffkd_specs", "encfm_specs", "meta_specs", "meta_bn_specs", "encfm_fixed_steps", "head_modules", "student_specs",
           "teacher_specs", "bn_buffer_specs", "fused_groups", "field"]
