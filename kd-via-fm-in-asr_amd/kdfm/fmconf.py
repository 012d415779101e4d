"""The FlowMatchingModule's "conformer" meta-encoder on the engine (kdfm/fmmeta.py drives the chain).

Reference: asr_train.py ConformerEncoder (:1000-1020) = input_proj Linear(Cs+E -> Cs) and 4
ConformerBlocks (:962-999) of width Cs with student_head_num heads, each
    x1 = x  + 0.5 * FF1(norm_ff1(x))          FeedForwardModule (:918-931): LN -> Linear(4Cs) -> SiLU -> drop
                                                                          -> Linear(Cs) -> drop
    x2 = x1 + MHA(mha_layer(x1))              nn.MultiheadAttention(batch_first, dropout) over the T frames
    x3 = x2 + Conv(x2)                        ConvModule (:932-961): LN -> pointwise_conv1 (Cs -> 2Cs, no GLU)
                                              -> depthwise k=31 (pad 15) -> BatchNorm1d (batch statistics) ->
                                              SiLU -> pointwise_conv2 (2Cs -> Cs) -> drop
    x4 = x3 + 0.5 * FF2(norm_ff2(x3))
    out = norm_final(x4)
Dropouts are the module's fixed 0.1 (ConformerEncoder's default, FlowMatchingModule passes none); the
engine runs them with the counter RNG when the config trains with dropout and at 0 in the parity
configuration (cfg.dropout == 0).  No padding masks: the reference feeds every frame (padded ones
included) to all of it, BatchNorm statistics included.

Kernels: LayerNorm fwd/bwd (norm.hip), the GEMM routes with SiLU / STORE_PRE / counter-RNG dropout /
residual epilogues (the FFN halves as in the unfused Conformer FFN path), the fused attention pair with a
zero positional table (attn_fused.hip / attn_bwd.hip bwd2), the k=31 depthwise conv with its fused
f64 BatchNorm sums and the BN+SiLU kernels (convmod.hip).  Every block evaluation keeps its own saves
(the chain evaluates the same parameters sum(S_i) times per step); the BatchNorm running statistics
are updated once per evaluation in forward order, as the reference's module calls are.
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K
from .mha import MhaShape, mha_bwd, mha_fwd

BLOCKS = 4
FF_MULT = 4
CONV_EXP = 2
CONV_K = 31
LN_EPS = 1e-5
BN_EPS = 1e-5
BN_MOMENTUM = 0.1
P_DROP = 0.1
SALT_META = 61
SITE_FF1_ACT, SITE_FF1_OUT, SITE_ATT, SITE_CONV_OUT, SITE_FF2_ACT, SITE_FF2_OUT = range(6)
ME = "flow_matching.meta_encoder."


def _stream(e, site):
    return SALT_META * (1 << 24) + e * 16 + site


def conformer_specs(Cs, E):
    """Parameters in the reference's named_parameters order (input_proj, then per block ff1.net.{0,1,4},
    norm_ff1, mha_layer, mha.{in_proj, out_proj}, conv_module.{layer_norm, pointwise_conv1, depthwise_conv,
    batch_norm, pointwise_conv2}, ff2.net.{0,1,4}, norm_ff2, norm_final)."""
    d, ff, c2 = Cs, FF_MULT * Cs, CONV_EXP * Cs
    s = [(ME + "input_proj.weight", (d, Cs + E)), (ME + "input_proj.bias", (d,))]
    for l in range(BLOCKS):
        p = f"{ME}layers.{l}."

        def ffm(name):
            return [(p + name + ".net.0.weight", (d,)), (p + name + ".net.0.bias", (d,)),
                    (p + name + ".net.1.weight", (ff, d)), (p + name + ".net.1.bias", (ff,)),
                    (p + name + ".net.4.weight", (d, ff)), (p + name + ".net.4.bias", (d,))]

        s += ffm("ff1")
        s += [(p + "norm_ff1.weight", (d,)), (p + "norm_ff1.bias", (d,)),
              (p + "mha_layer.weight", (d,)), (p + "mha_layer.bias", (d,)),
              (p + "mha.in_proj_weight", (3 * d, d)), (p + "mha.in_proj_bias", (3 * d,)),
              (p + "mha.out_proj.weight", (d, d)), (p + "mha.out_proj.bias", (d,)),
              (p + "conv_module.layer_norm.weight", (d,)), (p + "conv_module.layer_norm.bias", (d,)),
              (p + "conv_module.pointwise_conv1.weight", (c2, d, 1)), (p + "conv_module.pointwise_conv1.bias", (c2,)),
              (p + "conv_module.depthwise_conv.weight", (c2, 1, CONV_K)),
              (p + "conv_module.depthwise_conv.bias", (c2,)),
              (p + "conv_module.batch_norm.weight", (c2,)), (p + "conv_module.batch_norm.bias", (c2,)),
              (p + "conv_module.pointwise_conv2.weight", (d, c2, 1)), (p + "conv_module.pointwise_conv2.bias", (d,))]
        s += ffm("ff2")
        s += [(p + "norm_ff2.weight", (d,)), (p + "norm_ff2.bias", (d,)),
              (p + "norm_final.weight", (d,)), (p + "norm_final.bias", (d,))]
    return s


def bn_buffer_specs(Cs):
    c2 = CONV_EXP * Cs
    out = []
    for l in range(BLOCKS):
        p = f"{ME}layers.{l}.conv_module.batch_norm."
        out += [(p + "running_mean", (c2,)), (p + "running_var", (c2,))]
    return out


class _Saves:
    """One block evaluation's saved activations (n rows)."""

    def __init__(self, n, d, B, H, T, dev):
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        ff, c2 = FF_MULT * d, CONV_EXP * d
        for k in ("y1", "y2", "x1", "y3", "o", "x2", "y4", "x3", "y5", "y6", "x4", "out"):
            setattr(self, k, f(n, d))
        for k in ("m1", "r1", "m2", "r2", "m3", "r3", "m4", "r4", "m5", "r5", "m6", "r6", "m7", "r7"):
            setattr(self, k, f(n))
        self.h, self.a, self.h2, self.a2 = f(n, ff), f(n, ff), f(n, ff), f(n, ff)
        self.qkv, self.q = f(n, 3 * d), f(n, d)
        self.att = None   # kdfm/mha.py saves for the current math mode
        self.g, self.y, self.z = f(n, c2), f(n, c2), f(n, c2)
        self.bmean, self.brstd = f(c2), f(c2)
        self.stats = torch.empty(2 * c2, device=dev, dtype=torch.float64)


class ConformerMeta:
    """Saves and backward scratch of the conformer meta-encoder for `evals` meta-encoder evaluations."""

    def __init__(self, cfg, n, B, T, evals, dev):
        d = cfg.d_student
        H = cfg.heads_student
        if d % H or (d // H) % 4 or d // H > 64:
            raise ValueError(f"conformer meta-encoder: {d} channels over {H} heads needs a head dim that is a "
                             "multiple of 4 and <= 64 (the fused attention kernels)")
        self.d, self.H, self.B, self.T, self.n = d, H, B, T, n
        self.p = P_DROP if cfg.dropout > 0 else 0.0
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        self.xin = f(evals, n, d)
        self.sv = [_Saves(n, d, B, H, T, dev) for _ in range(evals * BLOCKS)]
        ff, c2 = FF_MULT * d, CONV_EXP * d
        self.dev = dev
        self.mha = None
        # backward scratch (shared by every evaluation: the backward runs them one after another)
        self.dA, self.dB, self.dC, self.dD = f(n, d), f(n, d), f(n, d), f(n, d)
        self.dff = f(n, ff)
        self.dc2a, self.dc2b = f(n, c2), f(n, c2)
        self.dqkv = f(n, 3 * d)
        self.red = torch.empty(2 * c2, device=dev, dtype=torch.float64)
        self._t1, self._t2, self._t3 = f(n, d), f(n, d), f(n, d)
        self._g0, self._g1 = f(n, d), f(n, d)

    def attention(self):
        """kdfm/mha.py buffers for the current math mode (re-made when the mode changes)."""
        fused = K.get_math() == "bf16"
        if self.mha is None or self.mha.fused != fused:
            self.mha = MhaShape(self.B, self.H, self.T, self.d, self.dev)
            for s in self.sv:
                s.att = self.mha.saves(self.dev)
        return self.mha


def _block_fwd(cm, P, pre, s, x, e, seed, bn_running, train):
    d, H, B, T = cm.d, cm.H, cm.B, cm.T
    c2 = CONV_EXP * d
    p = cm.p if train else 0.0
    # FF1 half step: x1 = x + 0.5 drop(W2 drop(silu(W1 LN(LN(x)))))
    K.layernorm_fwd(x, P[pre + "norm_ff1.weight"], P[pre + "norm_ff1.bias"], s.y1, s.m1, s.r1, LN_EPS)
    K.layernorm_fwd(s.y1, P[pre + "ff1.net.0.weight"], P[pre + "ff1.net.0.bias"], s.y2, s.m2, s.r2, LN_EPS)
    K.linear(s.y2, P[pre + "ff1.net.1.weight"], P[pre + "ff1.net.1.bias"], s.a, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE,
             Cpre=s.h, dropout_p=p, seed=seed, rng_stream=_stream(e, SITE_FF1_ACT))
    K.linear(s.a, P[pre + "ff1.net.4.weight"], P[pre + "ff1.net.4.bias"], s.x1, epi=_lib.EPI_RESID, R=x, rscale=0.5,
             dropout_p=p, seed=seed, rng_stream=_stream(e, SITE_FF1_OUT))
    # MHA: x2 = x1 + out_proj(softmax(q k^T / sqrt(dk)) v) on LN(x1)
    K.layernorm_fwd(s.x1, P[pre + "mha_layer.weight"], P[pre + "mha_layer.bias"], s.y3, s.m3, s.r3, LN_EPS)
    K.linear(s.y3, P[pre + "mha.in_proj_weight"], P[pre + "mha.in_proj_bias"], s.qkv)
    mha_fwd(cm.attention(), s.att, s.qkv, s.q, s.o, p, seed, _stream(e, SITE_ATT))
    K.linear(s.o, P[pre + "mha.out_proj.weight"], P[pre + "mha.out_proj.bias"], s.x2, epi=_lib.EPI_RESID, R=s.x1,
             rscale=1.0)
    # conv module: x3 = x2 + drop(pw2(silu(BN(dwconv(pw1(LN(x2)))))))
    K.layernorm_fwd(s.x2, P[pre + "conv_module.layer_norm.weight"], P[pre + "conv_module.layer_norm.bias"], s.y4, s.m4,
                    s.r4, LN_EPS)
    K.linear(s.y4, P[pre + "conv_module.pointwise_conv1.weight"].view(c2, d), P[pre + "conv_module.pointwise_conv1.bias"],
             s.g)
    s.stats.zero_()
    K.dwconv_fwd(s.g, P[pre + "conv_module.depthwise_conv.weight"].view(c2, CONV_K),
                 P[pre + "conv_module.depthwise_conv.bias"], s.y, s.stats, B, T, c2, CONV_K)
    bn = f"{ME}layers.{pre.split('.')[-2]}.conv_module.batch_norm."
    rm, rv = (bn_running[bn + "running_mean"], bn_running[bn + "running_var"]) if bn_running is not None else (None, None)
    if train and rm is not None:
        K.bn_finalize_running(s.stats, rm, rv, s.bmean, s.brstd, c2, cm.n, BN_EPS, BN_MOMENTUM)
    else:
        K.bn_finalize(s.stats, rm, rv, s.bmean, s.brstd, c2, cm.n, BN_EPS)
    K.bn_silu_fwd(s.y, s.bmean, s.brstd, P[pre + "conv_module.batch_norm.weight"], P[pre + "conv_module.batch_norm.bias"],
                  s.z)
    K.linear(s.z, P[pre + "conv_module.pointwise_conv2.weight"].view(d, c2), P[pre + "conv_module.pointwise_conv2.bias"],
             s.x3, epi=_lib.EPI_RESID, R=s.x2, rscale=1.0, dropout_p=p, seed=seed,
             rng_stream=_stream(e, SITE_CONV_OUT))
    # FF2 half step and the final LayerNorm
    K.layernorm_fwd(s.x3, P[pre + "norm_ff2.weight"], P[pre + "norm_ff2.bias"], s.y5, s.m5, s.r5, LN_EPS)
    K.layernorm_fwd(s.y5, P[pre + "ff2.net.0.weight"], P[pre + "ff2.net.0.bias"], s.y6, s.m6, s.r6, LN_EPS)
    K.linear(s.y6, P[pre + "ff2.net.1.weight"], P[pre + "ff2.net.1.bias"], s.a2, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE,
             Cpre=s.h2, dropout_p=p, seed=seed, rng_stream=_stream(e, SITE_FF2_ACT))
    K.linear(s.a2, P[pre + "ff2.net.4.weight"], P[pre + "ff2.net.4.bias"], s.x4, epi=_lib.EPI_RESID, R=s.x3,
             rscale=0.5, dropout_p=p, seed=seed, rng_stream=_stream(e, SITE_FF2_OUT))
    K.layernorm_fwd(s.x4, P[pre + "norm_final.weight"], P[pre + "norm_final.bias"], s.out, s.m7, s.r7, LN_EPS)
    return s.out


def conformer_fwd(cm, P, k, slab, seed, bn_running, train):
    """v = ConformerEncoder([x | e]) for evaluation k of the chain; returns the (n, Cs) output tensor."""
    x = cm.xin[k]
    K.linear(slab, P[ME + "input_proj.weight"], P[ME + "input_proj.bias"], x)
    for l in range(BLOCKS):
        x = _block_fwd(cm, P, f"{ME}layers.{l}.", cm.sv[k * BLOCKS + l], x, k * BLOCKS + l, seed, bn_running, train)
    return x


def _ff_bwd(cm, P, G, pre, name, norm, s_x, y_in, y_ln, m_in, r_in, m_ln, r_ln, h, a, dout, dres, dx, e, site_act,
            site_out, seed):
    """x_out = x + 0.5 drop(W2 drop(silu(W1 LN_net(LN_norm(x)) + b1)) + b2): dx = d x (+ dres from the residual)."""
    p = cm.p
    dl = cm.dB
    K.dropout(dout, dl, p, 0.5, seed, _stream(e, site_out))
    K.linear_dw(dl, a, G[pre + name + ".net.4.weight"], db=G[pre + name + ".net.4.bias"])
    K.linear_dx(dl, P[pre + name + ".net.4.weight"], cm.dff, epi=_lib.EPI_DSILU, aux=h, dropout_p=p, seed=seed,
                rng_stream=_stream(e, site_act))
    K.linear_dw(cm.dff, y_ln, G[pre + name + ".net.1.weight"], db=G[pre + name + ".net.1.bias"])
    K.linear_dx(cm.dff, P[pre + name + ".net.1.weight"], cm.dC)
    # LN_net backward (input y_in = LN_norm(x)), then LN_norm backward with the residual gradient
    K.layernorm_bwd(cm.dC, y_in, P[pre + name + ".net.0.weight"], m_ln, r_ln, cm.dD, G[pre + name + ".net.0.weight"],
                    G[pre + name + ".net.0.bias"])
    K.layernorm_bwd(cm.dD, s_x, P[pre + norm + ".weight"], m_in, r_in, dx, G[pre + norm + ".weight"],
                    G[pre + norm + ".bias"], dres=dres)


def _block_bwd(cm, P, G, pre, s, x, dout, dx, e, seed):
    """dout = d loss / d block output (n, d) -> dx = d loss / d block input x (may alias nothing in s)."""
    d, H, B, T = cm.d, cm.H, cm.B, cm.T
    c2 = CONV_EXP * d
    p = cm.p
    # norm_final
    dx4 = cm.dA
    K.layernorm_bwd(dout, s.x4, P[pre + "norm_final.weight"], s.m7, s.r7, dx4, G[pre + "norm_final.weight"],
                    G[pre + "norm_final.bias"])
    # FF2 (residual x3)
    dx3 = cm._t3
    _ff_bwd(cm, P, G, pre, "ff2", "norm_ff2", s.x3, s.y5, s.y6, s.m5, s.r5, s.m6, s.r6, s.h2, s.a2, dx4, dx4, dx3, e,
            SITE_FF2_ACT, SITE_FF2_OUT, seed)
    # conv module (residual x2)
    dpw2 = cm.dB
    K.dropout(dx3, dpw2, p, 1.0, seed, _stream(e, SITE_CONV_OUT))
    W2 = P[pre + "conv_module.pointwise_conv2.weight"].view(d, c2)
    K.linear_dw(dpw2, s.z, G[pre + "conv_module.pointwise_conv2.weight"].view(d, c2),
                db=G[pre + "conv_module.pointwise_conv2.bias"])
    K.linear_dx(dpw2, W2, cm.dc2a)
    K.bn_silu_bwd(cm.dc2a, s.y, s.bmean, s.brstd, P[pre + "conv_module.batch_norm.weight"],
                  P[pre + "conv_module.batch_norm.bias"], cm.red, cm.dc2b, G[pre + "conv_module.batch_norm.weight"],
                  G[pre + "conv_module.batch_norm.bias"], batch_stats=True)
    K.dwconv_bwd(cm.dc2b, s.g, P[pre + "conv_module.depthwise_conv.weight"].view(c2, CONV_K), cm.dc2a,
                 G[pre + "conv_module.depthwise_conv.weight"].view(c2, CONV_K), G[pre + "conv_module.depthwise_conv.bias"],
                 B, T, c2, CONV_K)
    W1 = P[pre + "conv_module.pointwise_conv1.weight"].view(c2, d)
    K.linear_dw(cm.dc2a, s.y4, G[pre + "conv_module.pointwise_conv1.weight"].view(c2, d),
                db=G[pre + "conv_module.pointwise_conv1.bias"])
    K.linear_dx(cm.dc2a, W1, cm.dC)
    dx2 = cm._t2
    K.layernorm_bwd(cm.dC, s.x2, P[pre + "conv_module.layer_norm.weight"], s.m4, s.r4, dx2,
                    G[pre + "conv_module.layer_norm.weight"], G[pre + "conv_module.layer_norm.bias"], dres=dx3)
    # MHA (residual x1)
    K.linear_dw(dx2, s.o, G[pre + "mha.out_proj.weight"], db=G[pre + "mha.out_proj.bias"])
    do = cm.dB
    K.linear_dx(dx2, P[pre + "mha.out_proj.weight"], do)
    mha_bwd(cm.attention(), s.att, s.qkv, s.q, s.o, do, cm.dqkv, p, seed, _stream(e, SITE_ATT))
    K.linear_dw(cm.dqkv, s.y3, G[pre + "mha.in_proj_weight"], db=G[pre + "mha.in_proj_bias"])
    K.linear_dx(cm.dqkv, P[pre + "mha.in_proj_weight"], cm.dC)
    dx1 = cm._t1
    K.layernorm_bwd(cm.dC, s.x1, P[pre + "mha_layer.weight"], s.m3, s.r3, dx1, G[pre + "mha_layer.weight"],
                    G[pre + "mha_layer.bias"], dres=dx2)
    # FF1 (residual x)
    _ff_bwd(cm, P, G, pre, "ff1", "norm_ff1", x, s.y1, s.y2, s.m1, s.r1, s.m2, s.r2, s.h, s.a, dx1, dx1, dx, e,
            SITE_FF1_ACT, SITE_FF1_OUT, seed)


def conformer_bwd(cm, P, G, k, slab, dv, dembed, seed):
    """dembed (n, Cs+E) = d loss / d [x | e] of evaluation k given dv = d loss / d v; parameter gradients
    accumulated into G."""
    g_out = cm._g0
    K.axpby(dv, None, g_out, 1.0, 0.0)
    for l in range(BLOCKS - 1, -1, -1):
        e = k * BLOCKS + l
        x = cm.xin[k] if l == 0 else cm.sv[e - 1].out
        dx = cm._g1
        _block_bwd(cm, P, G, f"{ME}layers.{l}.", cm.sv[e], x, g_out, dx, e, seed)
        g_out, cm._g1 = dx, g_out
        cm._g0 = g_out
    K.linear_dw(g_out, slab, G[ME + "input_proj.weight"], db=G[ME + "input_proj.bias"])
    K.linear_dx(g_out, P[ME + "input_proj.weight"], dembed)



__all__ = ["ConformerMeta", "conformer_specs", "bn_buffer_specs", "conformer_fwd", "conformer_bwd", "BLOCKS"]
