"""Drop-in NeMo-signature modules over libkdfm (the host side of the boundary).

The reference reaches its hot path through NeMo's module contract, not a C ABI:
asr_train_diffm.py:606-828 calls `preprocessor(input_signal=, length=)`, `spec_augmentation(
input_spec=, length=)`, `encoder(audio_signal=, length=)` with forward hooks on `encoder.layers[i]`,
`decoder(encoder_output=)`, `loss(log_probs=, targets=, input_lengths=, target_lengths=)` and the
ver5 heads `tae / sproj / adapter / denoiser / fm_latent` on (B, C, T) tensors.  The classes below
keep those names, argument names, shapes, return tuples and state-dict keys (Appendix A.10); their
forwards are torch.autograd.Functions whose forward and backward run libkdfm kernels, so the
reference's training_step code runs unchanged on top of them.  DistilFlowMatchingCTCModelBPE
mirrors the reference class (asr_train_diffm.py:500-838) and can hand its weights to the fused
Ver5Engine for the graph-captured production step.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from .overlap import WGRAD
from .config import Ver5Config, encoder_specs, sub_stages
from .conformer import EncoderShapes, compute_lengths, layer_backward, layer_forward, make_workspace, \
    subsampling_backward, subsampling_forward
from .frontend import FrontendConsts, frontend_forward, mel_frames, specaugment_

_SALT = 11


def _dev_check(t):
    if not t.is_cuda:
        raise _lib.KdfmError("kdfm modules run on the MI355X (HIP) device; move the module and inputs to 'cuda'")


def _tree_param(module: nn.Module, dotted: str, tensor: torch.Tensor):
    parts = dotted.split(".")
    m = module
    for p in parts[:-1]:
        if not hasattr(m, p) or not isinstance(getattr(m, p), nn.Module):
            setattr(m, p, nn.Module())
        m = getattr(m, p)
    m.register_parameter(parts[-1], nn.Parameter(tensor))


class _Flat(nn.Module):
    """Module whose parameters are views into ONE contiguous fp32 buffer (q|k|v adjacent), so the
    fused kernels see the same layout the engine uses; state-dict keys stay NeMo's."""

    def _flat_init(self, specs, device=None):
        device = device or torch.device("cpu")
        total = 0
        self._offsets = []
        for name, shape in specs:
            n = int(math.prod(shape)) if shape else 1
            self._offsets.append((name, total, n, shape))
            total += -(-n // 4) * 4
        self._flat = torch.zeros(total, device=device)
        for name, off, n, shape in self._offsets:
            _tree_param(self, name, self._flat[off:off + n].view(shape))
        self._specs = list(specs)

    def flat_params(self):
        return [self.get_parameter(name) for name, _ in self._specs]

    def _apply(self, fn, *a, **k):
        # .to()/.cuda() move parameters one by one; re-pack them into one buffer so the fused
        # q|k|v view (and any flat consumer) stays valid on the new device.
        out = super()._apply(fn, *a, **k)
        ps = self.flat_params()
        dev = ps[0].device
        total = self._flat.numel()
        flat = torch.zeros(total, device=dev, dtype=torch.float32)
        for (name, off, n, shape), prm in zip(self._offsets, ps):
            flat[off:off + n].copy_(prm.data.reshape(-1))
            prm.data = flat[off:off + n].view(shape)
        self._flat = flat
        return out

    def _P(self, params):
        P = {name: t for (name, _), t in zip(self._specs, params)}
        for name, t in list(P.items()):
            if name.endswith("self_attn.linear_q.weight"):
                base = name[: -len("linear_q.weight")]
                d = t.shape[0]
                P[base + "qkv.weight"] = t.as_strided((3 * d, d), (d, 1))
                P[base + "qkv.bias"] = P[base + "linear_q.bias"].as_strided((3 * d,), (1,))
        return P

    @staticmethod
    def _G(specs, device):
        total = sum(-(-int(math.prod(s) if s else 1) // 4) * 4 for _, s in specs)
        buf = torch.zeros(total, device=device)
        G, off = {}, 0
        for name, shape in specs:
            n = int(math.prod(shape)) if shape else 1
            G[name] = buf[off:off + n].view(shape)
            off += -(-n // 4) * 4
        for name in list(G):
            if name.endswith("self_attn.linear_q.weight"):
                base = name[: -len("linear_q.weight")]
                d = G[name].shape[0]
                G[base + "qkv.weight"] = G[name].as_strided((3 * d, d), (d, 1))
                G[base + "qkv.bias"] = G[base + "linear_q.bias"].as_strided((3 * d,), (1,))
        return G


# ------------------------------------------------------------------------------------------------
# Preprocessor / SpecAugment (audio_preprocessing.py:61-304, 443-553)
# ------------------------------------------------------------------------------------------------

class AudioToMelSpectrogramPreprocessor(nn.Module):
    def __init__(self, sample_rate=16000, window_size=0.025, window_stride=0.01, n_fft=512, features=80,
                 dither=1e-5, normalize="per_feature", window="hann", log=True, pad_to=0, pad_value=0.0,
                 preemph=0.97, **_):
        super().__init__()
        if normalize != "per_feature" or window != "hann" or not log or pad_to not in (0, None) or pad_value != 0.0:
            raise _lib.KdfmError("kdfm implements the Conformer-CTC recipe frontend (per_feature, hann, log, "
                                 "pad_to 0, pad_value 0)")
        self.cfg = Ver5Config(sample_rate=sample_rate, win=int(window_size * sample_rate),
                              hop=int(window_stride * sample_rate), n_fft=n_fft, nfilt=features, dither=dither,
                              preemph=preemph)
        c = FrontendConsts(self.cfg, "cpu")
        self.featurizer = nn.Module()
        self.featurizer.register_buffer("window", c.window)
        self.featurizer.register_buffer("fb", c.fb.unsqueeze(0))
        self.featurizer.register_buffer("dft_basis", c.basis, persistent=False)
        self.featurizer.register_buffer("fft_twiddle", c.twiddle, persistent=False)
        # the filterbank may be replaced by a checkpoint's: every filter over all bins (dense)
        self.featurizer.register_buffer("fb_lo", torch.zeros(features, dtype=torch.int32), persistent=False)
        self.featurizer.register_buffer("fb_hi", torch.full((features,), n_fft // 2 + 1, dtype=torch.int32),
                                        persistent=False)
        self.register_buffer("_seed", torch.zeros(1, dtype=torch.int64), persistent=False)

    @torch.no_grad()
    def forward(self, input_signal, length):
        _dev_check(input_signal)
        c = type("C", (), {})()
        f = self.featurizer
        c.window, c.fb, c.basis, c.twiddle, c.fb_lo, c.fb_hi = (f.window, f.fb[0].contiguous(), f.dft_basis,
                                                                f.fft_twiddle, f.fb_lo, f.fb_hi)
        B = input_signal.shape[0]
        mel_len = torch.empty(B, dtype=torch.int64, device=input_signal.device)
        K.subsample_lengths(length.to(torch.int64).contiguous(), mel_len, None, None, self.cfg.hop)
        dither = self.cfg.dither if self.training else 0.0
        if dither > 0:
            K.step_advance(None, self._seed)
        mel = frontend_forward(self.cfg, c, input_signal.float().contiguous(), length.to(torch.int64).contiguous(),
                               mel_len, dither=dither, seed=self._seed, rng_stream=_SALT)
        return mel.transpose(1, 2), mel_len


class SpectrogramAugmentation(nn.Module):
    def __init__(self, freq_masks=2, time_masks=5, freq_width=27, time_width=0.05, **_):
        super().__init__()
        self.cfg = Ver5Config(freq_masks=freq_masks, time_masks=time_masks, freq_width=freq_width,
                              time_width=time_width)
        self.register_buffer("_seed", torch.zeros(1, dtype=torch.int64), persistent=False)

    @torch.no_grad()
    def forward(self, input_spec, length):
        _dev_check(input_spec)
        if not self.training:
            return input_spec
        x = input_spec.transpose(1, 2).contiguous()
        K.step_advance(None, self._seed)
        specaugment_(self.cfg, x, length.to(torch.int64).contiguous(), self._seed, _SALT + 1)
        return x.transpose(1, 2)


# ------------------------------------------------------------------------------------------------
# ConformerEncoder (conformer_encoder.py:62-850) with hookable layers
# ------------------------------------------------------------------------------------------------

class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos_emb, lengths, mod, rm, rv, *params):
        P = mod._P(params)
        S = mod._shapes(x)
        out = torch.empty_like(x)
        save = torch.is_grad_enabled() or any(p.requires_grad for p in params) or x.requires_grad
        lctx = layer_forward(mod.cfg, S, P, "", mod.idx, x.view(S.rows, S.d), out.view(S.rows, S.d), pos_emb,
                             lengths, train=mod.training, seed=mod._seed, salt=_SALT + 2, save=True,
                             bn_update=(rm, rv), rm_batch=mod.training)
        ctx.lctx, ctx.mod, ctx.S, ctx.pos, ctx.lengths = lctx, mod, S, pos_emb, lengths
        ctx.params = params
        del save
        return out

    @staticmethod
    def backward(ctx, dout):
        mod, S = ctx.mod, ctx.S
        P = mod._P(ctx.params)
        G = _Flat._G(mod._specs, dout.device)
        dx = layer_backward(mod.cfg, S, P, G, "", mod.idx, ctx.lctx, dout.contiguous().view(S.rows, S.d), ctx.pos,
                            ctx.lengths, seed=mod._seed, salt=_SALT + 2)
        WGRAD.join()  # the returned grads are read by autograd as soon as this returns
        ctx.lctx = None
        grads = [G[name] for name, _ in mod._specs]
        return (dx.view_as(dout), None, None, None, None, None, *grads)


class ConformerLayer(_Flat):
    """One Conformer block; forward(x, att_mask, pos_emb, pad_mask) -> (B, T, d) as NeMo's, so the
    reference's register_forward_hook captures (asr_train_diffm.py:587-596) see the same tensors.
    The padding is taken from pad_mask (True = padded)."""

    def __init__(self, cfg: Ver5Config, d: int, h: int, idx: int, device=None):
        super().__init__()
        self.cfg, self.d, self.h, self.idx = cfg, d, h, idx
        all_specs = encoder_specs(cfg, d, h, "")
        pre = f"layers.{idx}."
        self._flat_init([(n[len(pre):], s) for n, s in all_specs if n.startswith(pre)], device)
        self.conv.batch_norm.register_buffer("running_mean", torch.zeros(d, device=device))
        self.conv.batch_norm.register_buffer("running_var", torch.ones(d, device=device))
        self.conv.batch_norm.register_buffer("num_batches_tracked", torch.zeros((), dtype=torch.int64, device=device))
        self.register_buffer("_seed", torch.zeros(1, dtype=torch.int64, device=device), persistent=False)

    def _shapes(self, x):
        B, T, _ = x.shape
        S = EncoderShapes(self.cfg, B, 4 * (T - 1) + 1, self.d, self.h)
        S.T, S.rows = T, B * T
        return S

    def forward(self, x, att_mask=None, pos_emb=None, pad_mask=None, cache_last_channel=None, cache_last_time=None):
        _dev_check(x)
        B, T, _ = x.shape
        if pad_mask is not None:
            lengths = (~pad_mask).sum(dim=1).to(torch.int64)
        else:
            lengths = torch.full((B,), T, dtype=torch.int64, device=x.device)
        if self.training:
            self.conv.batch_norm.num_batches_tracked += 1
        bn = self.conv.batch_norm
        return _LayerFn.apply(x.contiguous(), pos_emb.reshape(-1, self.d).contiguous(), lengths, self,
                              bn.running_mean, bn.running_var, *self.flat_params())


class _SubsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mel_btf, mel_len, len1, len2, mod, *params):
        P = mod._P(params)
        S = EncoderShapes(mod.cfg, mel_btf.shape[0], mel_btf.shape[1], mod.d, 1)
        P = {"pre_encode." + k: v for k, v in P.items()}
        x, sctx = subsampling_forward(mod.cfg, S, P, "", mel_btf.contiguous(), mel_len, len1, len2,
                                      train=mod.training, seed=mod._seed, salt=_SALT + 3, save=True, ws=mod._ws(S))
        ctx.sctx, ctx.S, ctx.mod, ctx.len1, ctx.params = sctx, S, mod, len1, params
        return x.view(S.B, S.T, S.d)

    @staticmethod
    def backward(ctx, dx):
        mod, S = ctx.mod, ctx.S
        G = _Flat._G(mod._specs, dx.device)
        Gp = {"pre_encode." + k: v for k, v in G.items()}
        Pp = {"pre_encode." + k: v for k, v in mod._P(ctx.params).items()}
        subsampling_backward(mod.cfg, S, Pp, Gp, "", ctx.sctx, dx.contiguous().view(S.rows, S.d),
                             ctx.len1, seed=mod._seed, salt=_SALT + 3, ws=mod._ws(S))
        WGRAD.join()
        return (None, None, None, None, None, *[G[n] for n, _ in mod._specs])


class ConvSubsampling(_Flat):
    """ConvSubsampling (conformer_encoder.py:381-390): 'striding' x4 (Appendix A.3) or 'dw_striding'
    (x2^n, depthwise-separable, optional causal padding; oracle/ver5.py subsampling_dw_striding).
    forward(x (B, T, feat_in), lengths) -> ((B, T', d), lengths')."""

    def __init__(self, cfg: Ver5Config, d: int, device=None):
        super().__init__()
        self.cfg, self.d = cfg, d
        self._flat_init([(n[len("pre_encode."):], s) for n, s in encoder_specs(cfg, d, 1, "")
                         if n.startswith("pre_encode.")], device)
        self._wsd = {}
        self.register_buffer("_seed", torch.zeros(1, dtype=torch.int64, device=device), persistent=False)

    def _ws(self, S):
        if S.F2 not in self._wsd:
            self._wsd[S.F2] = make_workspace(S, self._flat.device)
        return self._wsd[S.F2]

    def forward(self, x, lengths):
        _dev_check(x)
        B = x.shape[0]
        lengths = lengths.to(torch.int64).contiguous()
        len1 = torch.empty(B, dtype=torch.int64, device=x.device)
        len2 = torch.empty_like(len1)
        # lengths are mel frames here (hop 1): calc_length per stage
        len1, len2 = compute_lengths(self.cfg, lengths, torch.empty_like(len1), len1, len2, 1)
        y = _SubsampleFn.apply(x, lengths, len1, len2, self, *self.flat_params())
        return y, len2


class RelPositionalEncoding(nn.Module):
    def __init__(self, d_model: int, xscale=None):
        super().__init__()
        self.d_model, self.xscale = d_model, xscale
        self._tables = {}

    def forward(self, x, cache_len=0):
        T = x.shape[1]
        key = (T, x.device)
        if key not in self._tables:
            pe = torch.empty(2 * T - 1, self.d_model, device=x.device)
            K.relpos_table(T, self.d_model, pe)
            self._tables[key] = pe
        return x, self._tables[key].unsqueeze(0)


class ConformerEncoder(nn.Module):
    """NeMo ConformerEncoder API: forward(audio_signal (B, feat_in, T), length) -> ((B, d, T'), lengths).
    The x*sqrt(d) scaling (xscaling) and pre-encoder dropout are fused into pre_encode's output GEMM."""

    def __init__(self, feat_in=80, n_layers=16, d_model=176, n_heads=4, subsampling="striding",
                 subsampling_factor=4, subsampling_conv_channels=-1, causal_downsampling=False, ff_expansion_factor=4,
                 self_attention_model="rel_pos", conv_kernel_size=31, dropout=0.1, dropout_pre_encoder=0.1,
                 dropout_emb=0.0, dropout_att=0.1, xscaling=True, untie_biases=True, pos_emb_max_len=5000,
                 conv_norm_type="batch_norm", device=None, init_seed=0, **_):
        super().__init__()
        if self_attention_model != "rel_pos" or conv_norm_type != "batch_norm" or not untie_biases \
                or (subsampling == "striding" and subsampling_conv_channels not in (-1, d_model)):
            raise _lib.KdfmError("kdfm ConformerEncoder implements the Conformer-CTC / FastConformer recipes "
                                 "(rel_pos, batch_norm conv, untied biases)")
        self.cfg = Ver5Config(nfilt=feat_in, n_layers=n_layers, ff_expansion=ff_expansion_factor,
                              conv_kernel=conv_kernel_size, dropout=dropout, dropout_pre=dropout_pre_encoder,
                              dropout_att=dropout_att, subsampling=subsampling, subsampling_factor=subsampling_factor,
                              subsampling_conv_channels=subsampling_conv_channels,
                              causal_downsampling=causal_downsampling, xscaling=xscaling)
        sub_stages(self.cfg)   # validates the subsampling choice
        self.d_model, self.n_heads = d_model, n_heads
        self._feat_out = d_model
        self.pre_encode = ConvSubsampling(self.cfg, d_model, device)
        self.pos_enc = RelPositionalEncoding(d_model, math.sqrt(d_model) if xscaling else None)
        self.layers = nn.ModuleList([ConformerLayer(self.cfg, d_model, n_heads, i, device) for i in range(n_layers)])
        self.register_buffer("_seed", torch.zeros(1, dtype=torch.int64, device=device), persistent=False)
        self.init_weights(init_seed)

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Seeded random init (the same scheme the fused engine uses; kdfm.store.init_uniform)."""
        from .store import init_uniform
        specs = encoder_specs(self.cfg, self.d_model, self.n_heads, "")
        vals = init_uniform(specs, seed)
        for name, _ in specs:
            self.get_parameter(name).copy_(vals[name])

    def forward(self, audio_signal, length=None):
        _dev_check(audio_signal)
        if length is None:
            length = torch.full((audio_signal.shape[0],), audio_signal.shape[-1], dtype=torch.int64,
                                device=audio_signal.device)
        if self.training:
            K.step_advance(None, self._seed)
        for m in [self.pre_encode] + list(self.layers):
            m._seed = self._seed
        x, length = self.pre_encode(audio_signal.transpose(1, 2), length)
        x, pos_emb = self.pos_enc(x)
        T = x.shape[1]
        pad_mask = torch.arange(T, device=x.device).expand(x.shape[0], T) >= length.unsqueeze(1)
        for layer in self.layers:
            x = layer(x=x, att_mask=None, pos_emb=pos_emb, pad_mask=pad_mask)
        return x.transpose(1, 2), length


# ------------------------------------------------------------------------------------------------
# Decoder + CTC (conv_asr.py:407-505; losses/ctc.py:25-82)
# ------------------------------------------------------------------------------------------------

class _DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc_btd, W, b):
        B, T, d = enc_btd.shape
        Cn = W.shape[0]
        x = enc_btd.contiguous().view(B * T, d)
        logits = torch.empty(B * T, Cn, device=x.device)
        K.linear(x, W.view(Cn, d), b, logits)
        lp = torch.empty_like(logits)
        K.log_softmax(logits, lp)
        ctx.save_for_backward(x, W, lp)
        return lp.view(B, T, Cn)

    @staticmethod
    def backward(ctx, dlp):
        x, W, lp = ctx.saved_tensors
        Cn, d = W.shape[0], x.shape[1]
        g = torch.empty_like(lp)
        K.log_softmax_bwd(dlp.contiguous().view_as(lp), lp, g)
        dW = torch.zeros(Cn, d, device=x.device)
        db = torch.zeros(Cn, device=x.device)
        K.linear_dw(g, x, dW, db=db)
        dx = torch.empty_like(x)
        K.linear_dx(g, W.view(Cn, d), dx)
        return dx.view(dlp.shape[0], dlp.shape[1], d), dW.view_as(W), db


class ConvASRDecoder(nn.Module):
    def __init__(self, feat_in, num_classes, vocabulary=None, add_blank=True, device=None, **_):
        super().__init__()
        self._feat_in = feat_in
        self._num_classes = num_classes + 1 if add_blank else num_classes
        self.decoder_layers = nn.Sequential(nn.Conv1d(feat_in, self._num_classes, kernel_size=1, bias=True))
        if device is not None:
            self.to(device)
        self.temperature = 1.0

    def forward(self, encoder_output):
        _dev_check(encoder_output)
        conv = self.decoder_layers[0]
        lp = _DecoderFn.apply(encoder_output.transpose(1, 2), conv.weight, conv.bias)
        if self.temperature != 1.0:
            raise _lib.KdfmError("decoder temperature != 1 is not on the training path")
        return lp


class _CTCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_probs, targets, in_len, tgt_len, blank, zero_inf):
        B, T, Cn = log_probs.shape
        lp = log_probs.contiguous()
        Umax = max(1, targets.shape[1])
        aws = torch.empty(B * T * (2 * Umax + 1), device=lp.device)
        bws = torch.empty_like(aws)
        nll = torch.empty(B, device=lp.device)
        grad = torch.empty(B * T, Cn, device=lp.device)
        K.ctc_loss(lp.view(B * T, Cn), targets.to(torch.int64).contiguous(), in_len.to(torch.int64).contiguous(),
                   tgt_len.to(torch.int64).contiguous(), aws, bws, nll, grad, B, T, Cn, blank, 1.0, zero_inf)
        ctx.save_for_backward(grad)
        ctx.shape = (B, T, Cn)
        return nll

    @staticmethod
    def backward(ctx, dnll):
        (grad,) = ctx.saved_tensors
        B, T, Cn = ctx.shape
        # torch CTCLoss convention: d/d log_probs = (exp(lp) - posterior) * dnll[b]
        out = torch.empty(B, T, Cn, device=grad.device)
        K.rowscale(grad, out, dnll.contiguous(), T)
        return out, None, None, None, None, None


class _ReduceFn(torch.autograd.Function):
    """scale * sum(x) on device (colsum kernel), backward broadcasts the upstream scalar."""

    @staticmethod
    def forward(ctx, x, scale):
        out = torch.empty(1, device=x.device)
        K.colsum(x.contiguous().view(-1, 1), out, scale=scale, accumulate=False)
        ctx.n, ctx.scale = x.numel(), scale
        ctx.shape = x.shape
        return out.view(())

    @staticmethod
    def backward(ctx, g):
        ones = torch.empty(ctx.n, device=g.device)
        K.fill(ones, 1.0)
        out = torch.empty_like(ones)
        K.rowscale(ones.view(-1, 1), out.view(-1, 1), g.reshape(1).contiguous(), ctx.n, ctx.scale)
        return out.view(ctx.shape), None


class CTCLoss(nn.Module):
    """NeMo CTCLoss(num_classes, zero_infinity, reduction='mean_batch') (losses/ctc.py:25-82)."""

    def __init__(self, num_classes, zero_infinity=True, reduction="mean_batch"):
        super().__init__()
        if reduction not in ("mean_batch", "none", "sum"):
            raise _lib.KdfmError("reduction must be mean_batch, none or sum")
        self._blank = num_classes
        self.zero_infinity = zero_infinity
        self.config_reduction = reduction

    def forward(self, log_probs, targets, input_lengths, target_lengths):
        _dev_check(log_probs)
        nll = _CTCFn.apply(log_probs, targets, input_lengths, target_lengths, self._blank, int(self.zero_infinity))
        if self.config_reduction == "none":
            return nll
        return _ReduceFn.apply(nll, 1.0 / nll.numel() if self.config_reduction == "mean_batch" else 1.0)


__all__ = ["AudioToMelSpectrogramPreprocessor", "SpectrogramAugmentation", "ConformerEncoder", "ConformerLayer",
           "ConvSubsampling", "ConvASRDecoder", "CTCLoss", "mel_frames"]
