"""Encoder-level flow matching with the "cnn" and "swin" meta-encoders (fixed step counts) on the engine.

Reference: asr_train.py FlowMatchingModule (:1220-1377) with flow_cfg["meta_encoder_type"] = "cnn"
(:1251-1257: Conv1d(Cs+E, Cs, 3, pad 1) -> ReLU -> Conv1d(Cs, Cs, 1)) or "swin" (:1258-1259,
SwinTransformerEncoder :844-866: nn.MultiheadAttention over the frames of each utterance with
student_head_num heads, then Linear(Cs+E, Cs) -> ReLU -> Linear(Cs, Cs)); the flowkd_<meta>_linear_*
launchers.  Per hooked layer i with S_i steps: x_0 = s_i; for k = S..1 (t = k/S) the meta-encoder reads
[x | time_embed(t)] and x <- x - v / S; the loss regresses the teacher's features from
noise_scheduled_x = ca(S) s_i + cv(S) v_last through shape_transformation_function (MSE); the
decoder reads the last layer's x_S (:666).

Engine layout (rows = B*T frames, channels-last): every step's meta-encoder input [x_j | e_j] lives in
one (rows, Cs+E) slab of a resident (sum S_i, rows, Cs+E) buffer, so x_{j+1} is written by the last
GEMM's residual epilogue straight into the next slab's first Cs columns (no separate x tensors), and
the backward re-reads the slabs as its saved activations.  The cnn's k=3 conv is the implicit-GEMM
conv3 (LD_CONV taps across utterance borders zero-padded, as Conv1d's pad=1); the swin's attention is
kdfm/mha.py (the fused attention pair in bf16 math, the exact-f32 unfused form in parity math): plain
softmax(q k^T / sqrt(dk)) v -- nn.MultiheadAttention without masks (every frame, padded ones included,
as the reference).  Only fixed step counts (sampling_steps_per_layer): the
router's per-utterance counts would put a device->host sync on the step to drive the per-step
launches; with meta "mlp" the dynamic router path is kdfm/encfm.py.  Step counts: config.encfm_fixed_steps
(sampling_steps_per_layer, else --flow_steps for every layer).  Parity: tests/golden/
kd_encfm_meta.npz (the reference's own classes).
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K
from .config import encfm_fixed_steps
from .encfm import schedule_coeffs
from .mha import mha_bwd, mha_fwd

META_TYPES = ("mlp", "cnn", "swin", "conformer")


class MetaFMWorkspace:
    """Per-(B, T) resident buffers for the meta-encoder chain (fixed steps, so every size is static)."""

    def __init__(self, cfg, B, T, dev):
        if cfg.encfm_meta not in ("cnn", "swin", "conformer"):
            raise ValueError(f"MetaFMWorkspace is for the cnn / swin / conformer meta-encoders, got {cfg.encfm_meta!r}")
        L, Cs, Ct, E = cfg.n_layers, cfg.d_student, cfg.d_teacher, cfg.time_embed_dim
        if cfg.encfm_dynamic:
            raise ValueError("meta_encoder 'cnn' / 'swin' run with fixed step counts (encfm_dynamic=False)")
        steps = list(encfm_fixed_steps(cfg))
        Ci = Cs + E
        n = B * T
        self.meta, self.B, self.T, self.n, self.Ci = cfg.encfm_meta, B, T, n, Ci
        self.steps = steps
        self.base = [sum(steps[:i]) for i in range(L)]
        N = sum(steps)
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        self.embed = f(N, n, Ci)          # [x_j | e_j] per step (the backward's saved inputs)
        self.erow = f(N, E)               # time embedding of each step
        self.vl = f(n, Cs)                # v of the layer's last step
        self.nsx, self.dtr = f(L, n, Cs), f(L, n, Ct)
        self.xS, self.gxS = f(n, Cs), f(n, Cs)
        self.flow, self.rloss, self.mean_steps = f(L), torch.zeros(L, device=dev), f(L)
        self.mean_steps.copy_(torch.tensor([float(s) for s in steps]))
        self.stats = torch.zeros(4, device=dev)
        self.inv = 1.0 / (n * Ct)
        ca, cv, _, _ = schedule_coeffs(cfg)
        self.ca = [float(ca[s - 1]) for s in steps]
        self.cv = [float(cv[s - 1]) for s in steps]
        # backward scratch
        self.gx, self.dv, self.dnsx, self.dembed = f(n, Cs), f(n, Cs), f(n, Cs), f(n, Ci)
        if self.meta == "cnn":
            self.act = f(N, n, Cs)
            self.w0f, self.w0b, self.g0 = f(Cs, 3 * Ci), f(Ci, 3 * Cs), f(Cs, 3 * Ci)
            self.da = f(n, Cs)
        elif self.meta == "conformer":
            from .fmconf import ConformerMeta
            self.conf = ConformerMeta(cfg, n, B, T, N, dev)
        else:
            H = cfg.heads_student
            if Ci % H or (Ci // H) % 4 or Ci // H > 64:
                raise ValueError(f"swin meta-encoder: {Ci} channels over {H} heads needs a head dim that is a "
                                 "multiple of 4 and <= 64 (the fused attention kernels)")
            self.H = H
            self.qkv, self.q, self.o = f(N, n, 3 * Ci), f(N, n, Ci), f(N, n, Ci)
            self.ao, self.h = f(N, n, Ci), f(N, n, Cs)
            self.dpre, self.dao, self.do = f(n, Cs), f(n, Ci), f(n, Ci)
            self.dqkv = f(n, 3 * Ci)
            self.mha, self.att = None, None   # per-math attention buffers (kdfm/mha.py), made at first use
        self.dev = dev

    def attention(self):
        """The attention buffers for the current math mode (fused bf16 pair or exact-f32 unfused form)."""
        from .mha import MhaShape
        fused = K.get_math() == "bf16"
        if self.mha is None or self.mha.fused != fused:
            self.mha = MhaShape(self.B, self.H, self.T, self.Ci, self.dev)
            self.att = [self.mha.saves(self.dev) for _ in range(self.embed.shape[0])]
        return self.mha


def _names(meta):
    me = "flow_matching.meta_encoder."
    if meta == "conformer":
        return {}
    if meta == "cnn":
        return dict(w0=me + "0.weight", b0=me + "0.bias", w2=me + "2.weight", b2=me + "2.bias")
    return dict(win=me + "attn.in_proj_weight", bin=me + "attn.in_proj_bias", wo=me + "attn.out_proj.weight",
                bo=me + "attn.out_proj.bias", w1=me + "linear1.weight", b1=me + "linear1.bias",
                w2=me + "linear2.weight", b2=me + "linear2.bias")


def _meta_fwd(ws, P, nm, k, out, R, rscale, seed=None, bn_running=None, train=True):
    """One meta-encoder evaluation on slab k: out = v (R None) or R + rscale * v."""
    Cs = out.shape[1]
    x = ws.embed[k]
    epi = _lib.EPI_RESID if R is not None else 0
    if ws.meta == "conformer":
        from .fmconf import conformer_fwd
        v = conformer_fwd(ws.conf, P, k, x, seed, bn_running, train)
        if R is None:
            K.axpby(v, None, out, 1.0, 0.0)
        else:
            K.axpby(R, v, out, 1.0, rscale)
        return
    if ws.meta == "cnn":
        K.conv3(x, ws.w0f, P[nm["b0"]], ws.act[k], ws.T, epi=_lib.EPI_RELU)
        K.linear(ws.act[k], P[nm["w2"]].view(Cs, Cs), P[nm["b2"]], out, epi=epi, R=R, rscale=rscale)
        return
    K.linear(x, P[nm["win"]], P[nm["bin"]], ws.qkv[k])
    mha_fwd(ws.attention(), ws.att[k], ws.qkv[k], ws.q[k], ws.o[k], 0.0, None, 0)   # MHA dropout 0 (:847)
    K.linear(ws.o[k], P[nm["wo"]], P[nm["bo"]], ws.ao[k])
    K.linear(ws.ao[k], P[nm["w1"]], P[nm["b1"]], ws.h[k], epi=_lib.EPI_RELU)
    K.linear(ws.h[k], P[nm["w2"]], P[nm["b2"]], out, epi=epi, R=R, rscale=rscale)


def _meta_bwd(ws, P, G, nm, k, dv, dembed, seed=None):
    """dembed = d/d[x | e] of slab k's meta-encoder given dv; parameter gradients accumulated into G."""
    Cs = dv.shape[1]
    x = ws.embed[k]
    if ws.meta == "conformer":
        from .fmconf import conformer_bwd
        conformer_bwd(ws.conf, P, G, k, x, dv, dembed, seed)
        return
    if ws.meta == "cnn":
        K.linear_dw(dv, ws.act[k], G[nm["w2"]].view(Cs, Cs), db=G[nm["b2"]])
        K.linear_dx(dv, P[nm["w2"]].view(Cs, Cs), ws.da, epi=_lib.EPI_DRELU, aux=ws.act[k])
        K.conv3_dw(ws.da, x, ws.g0, ws.T, db=G[nm["b0"]])
        K.conv3(ws.da, ws.w0b, None, dembed, ws.T)
        return
    K.linear_dw(dv, ws.h[k], G[nm["w2"]], db=G[nm["b2"]])
    K.linear_dx(dv, P[nm["w2"]], ws.dpre, epi=_lib.EPI_DRELU, aux=ws.h[k])
    K.linear_dw(ws.dpre, ws.ao[k], G[nm["w1"]], db=G[nm["b1"]])
    K.linear_dx(ws.dpre, P[nm["w1"]], ws.dao)
    K.linear_dw(ws.dao, ws.o[k], G[nm["wo"]], db=G[nm["bo"]])
    K.linear_dx(ws.dao, P[nm["wo"]], ws.do)
    mha_bwd(ws.attention(), ws.att[k], ws.qkv[k], ws.q[k], ws.o[k], ws.do, ws.dqkv, 0.0, None, 0)
    K.linear_dw(ws.dqkv, x, G[nm["win"]], db=G[nm["bin"]])
    K.linear_dx(ws.dqkv, P[nm["win"]], dembed)


def meta_forward(cfg, P, sfeats, tfeats, ws: MetaFMWorkspace, *, seed=None, bn_running=None, train=True):
    """All layers' FM chains.  sfeats (L, B*T, Cs) / tfeats (L, B*T, Ct) hook outputs; returns ws.xS, the
    last layer's FM output.  ws.stats = [sum of flow losses, 0, total, mean steps] as encfm_forward.
    train=False: only the chains and x_S -- the flow losses are 0 as the reference's eval forward returns
    (asr_train.py:1363-1364), and noise_scheduled_x / the MSE / its gradient are not computed."""
    L, Cs, E, n = cfg.n_layers, cfg.d_student, cfg.time_embed_dim, ws.n
    fm = "flow_matching."
    nm = _names(ws.meta)
    if ws.meta == "cnn":
        K.convw_prep(P[nm["w0"]], fwd=ws.w0f)
    wte, bte = P[fm + "time_embed.weight"].view(1, E), P[fm + "time_embed.bias"].view(1, E)
    Wst, bst = P[fm + "shape_transformation_function.weight"], P[fm + "shape_transformation_function.bias"]
    K.fill(ws.flow, 0.0)
    for i in range(L):
        S, b0 = ws.steps[i], ws.base[i]
        s_i = sfeats[i].view(n, Cs)
        K.axpby(s_i, None, ws.embed[b0][:, :Cs], 1.0, 0.0)
        for j in range(S):
            k = b0 + j
            slab = ws.embed[k]
            K.axpby(wte, bte, ws.erow[k:k + 1], (S - j) / S, 1.0)          # time_embed(t), t = (S - j) / S
            K.axpby(ws.erow[k:k + 1].expand(n, E), None, slab[:, Cs:], 1.0, 0.0)
            if j < S - 1:   # x_{j+1} = x_j - v_j / S straight into the next slab
                _meta_fwd(ws, P, nm, k, ws.embed[k + 1][:, :Cs], slab[:, :Cs], -1.0 / S, seed, bn_running, train)
            else:
                _meta_fwd(ws, P, nm, k, ws.vl, None, 0.0, seed, bn_running, train)
        last = ws.embed[b0 + S - 1][:, :Cs]
        if i == L - 1:
            K.axpby(last, ws.vl, ws.xS, 1.0, -1.0 / S)
        if not train:   # the reference's loss is 0.0 outside training (asr_train.py:1363-1364): no nsx / MSE
            continue
        K.axpby(s_i, ws.vl, ws.nsx[i], ws.ca[i], ws.cv[i])              # noise_scheduled_x (:1366-1367)
        K.linear(ws.nsx[i], Wst, bst, ws.dtr[i], R=tfeats[i].view(n, -1), rscale=2.0 * ws.inv,
                 mse=(ws.flow[i:i + 1], ws.inv))                           # MSELoss and its gradient
    K.colsum(ws.flow.view(L, 1), ws.stats[0:1], accumulate=False)
    K.fill(ws.stats[1:2], 0.0)
    K.axpby(ws.stats[0:1].view(1, 1), None, ws.stats[2:3].view(1, 1), 1.0, 0.0)
    K.colsum(ws.mean_steps.view(L, 1), ws.stats[3:4], scale=1.0 / L, accumulate=False)
    return ws.xS


def meta_backward(cfg, P, G, ws: MetaFMWorkspace, dfeats, gxS, *, seed=None):
    """dfeats (L*B*T, Cs) (overwritten) = d loss / d s_i from the flow losses and gxS (d loss / d x_S of the
    last layer through the decoder); flow_matching.* parameter gradients accumulated into G."""
    L, Cs, E, n = cfg.n_layers, cfg.d_student, cfg.time_embed_dim, ws.n
    fm = "flow_matching."
    nm = _names(ws.meta)
    dfeats = dfeats.view(L, n, Cs)
    Wst = P[fm + "shape_transformation_function.weight"]
    gte_w, gte_b = G[fm + "time_embed.weight"].view(E), G[fm + "time_embed.bias"]
    if ws.meta == "cnn":
        K.convw_prep(P[nm["w0"]], bwd=ws.w0b)
        K.fill(ws.g0, 0.0)
    for i in range(L - 1, -1, -1):
        S, b0 = ws.steps[i], ws.base[i]
        K.linear_dx(ws.dtr[i], Wst, ws.dnsx)
        K.linear_dw(ws.dtr[i], ws.nsx[i], G[fm + "shape_transformation_function.weight"],
                    db=G[fm + "shape_transformation_function.bias"])
        have_gx = i == L - 1
        if have_gx:
            K.axpby(gxS, None, ws.gx, 1.0, 0.0)
        for j in range(S - 1, -1, -1):
            k = b0 + j
            if j == S - 1:   # v_last feeds noise_scheduled_x (cv) and, on the last layer, x_S (-1/S)
                K.axpby(ws.dnsx, ws.gx if have_gx else None, ws.dv, ws.cv[i], -1.0 / S if have_gx else 0.0)
            else:
                K.axpby(ws.gx, None, ws.dv, -1.0 / S, 0.0)
            _meta_bwd(ws, P, G, nm, k, ws.dv, ws.dembed, seed)
            if have_gx:
                K.axpby(ws.gx, ws.dembed[:, :Cs], ws.gx, 1.0, 1.0)
            else:
                K.axpby(ws.dembed[:, :Cs], None, ws.gx, 1.0, 0.0)
                have_gx = True
            K.colsum(ws.dembed[:, Cs:], gte_w, scale=(S - j) / S)
            K.colsum(ws.dembed[:, Cs:], gte_b)
        K.axpby(ws.gx, ws.dnsx, dfeats[i], 1.0, ws.ca[i])
    if ws.meta == "cnn":
        K.convw_grad(ws.g0, G[nm["w0"]])


__all__ = ["META_TYPES", "MetaFMWorkspace", "meta_forward", "meta_backward"]
