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

META_TYPES = ("mlp", "cnn", "swin", "conformer", "unet")


class MetaFMWorkspace:
    """Per-(B, T) resident buffers for the meta-encoder chain (fixed steps, so every size is static)."""

    def __init__(self, cfg, B, T, dev):
        if cfg.encfm_meta not in ("cnn", "swin", "conformer", "unet"):
            raise ValueError(f"MetaFMWorkspace is for the cnn / swin / conformer / unet meta-encoders, got "
                             f"{cfg.encfm_meta!r}")
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
        elif self.meta == "unet":
            self.unet = _UNetWs(cfg, B, T, N, dev)
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


class _UNetWs:
    """UNet1D (asr_train.py:880-917) buffers: per meta call k the concatenated up-path inputs of every level,
    cat[l][k] = [x part | skip of level l] (B * L_l rows; the skip is the down conv's output, written straight
    into its columns; the x part the bottleneck's (l = 4) or the next-deeper up's output, written by the fold,
    its rows past 2 L_{l+1} the reference's zero pad), and the last up's output (B * 2 L_1, base); the backward
    re-reads them (UNet1D has no nonlinearity: no other saves).  Scratch for the unfolded columns, the
    transposed convs' GEMM outputs and the gradients is shared by the calls."""

    def __init__(self, cfg, B, T, N, dev):
        from .config import UNET_LAYERS, unet_channels
        Cs, E, base = cfg.d_student, cfg.time_embed_dim, cfg.encfm_hidden
        nl = UNET_LAYERS
        L = [T]
        for _ in range(nl):
            L.append(L[-1] // 2)
        if 2 * L[1] != T:
            # the reference's update x - v / S then fails (asr_train.py:1358): UNet1D returns T - 1 frames
            raise ValueError(f"meta_encoder 'unet' needs an even frame count: UNet1D returns {2 * L[1]} frames for "
                             f"T={T} and the reference's x - velocity / S fails (RuntimeError: The size of tensor a "
                             f"({T}) must match the size of tensor b ({2 * L[1]}) at non-singleton dimension 1)")
        if any(v == 0 for v in L):
            raise ValueError(f"meta_encoder 'unet': T={T} frames is too short for {nl} stride-2 levels")
        if base % 4 or (Cs + E) % 4 or Cs % 4:
            raise ValueError("meta_encoder 'unet': channel counts must be multiples of 4")
        self.cin, self.cdown, self.ups = unet_channels(Cs, E, base, nl)
        self.L, self.nl, self.B, self.T = L, nl, B, T
        # x-part width per level l = 1..nl (index l): the bottleneck's at the deepest level, else the up output
        self.cx = [0] + [self.cdown[l] for l in range(1, nl)] + [self.cdown[-1]]
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        self.cat = [None] + [f(N, B * L[l], self.cx[l] + self.cdown[l - 1]) for l in range(1, nl + 1)]
        self.up_last = f(N, B * 2 * L[1], self.cdown[0])
        rows = max(B * L[i + 1] * 4 * self.cin[i] for i in range(nl))
        zrows = max(B * L[nl - j] * 4 * co for j, (_, co) in enumerate(self.ups))
        self.cols = f(max(rows, zrows))              # unfold / dZ scratch
        self.z = f(zrows)                            # transposed convs' GEMM outputs
        self.dcat = [None] + [f(B * L[l], self.cx[l] + self.cdown[l - 1]) for l in range(1, nl + 1)]
        self.dup = f(B * 2 * L[1], self.cdown[0])
        self.dbcols = f(max(B * 2 * L[l] * co for l, (_, co) in zip(range(nl, 0, -1), self.ups)))
        # weight layouts (kdfm_convw_prep) and GEMM-layout gradient accumulators
        self.wd = [f(self.cdown[i], 4 * self.cin[i]) for i in range(nl)]
        self.gd = [f(self.cdown[i], 4 * self.cin[i]) for i in range(nl)]
        cb = self.cdown[-1]
        self.wbf, self.wbb, self.gb = f(cb, 3 * cb), f(cb, 3 * cb), f(cb, 3 * cb)
        self.wu = [f(ci, 4 * co) for ci, co in self.ups]
        self.gu = [f(ci, 4 * co) for ci, co in self.ups]


def _names(meta):
    me = "flow_matching.meta_encoder."
    if meta in ("conformer", "unet"):
        return {}
    if meta == "cnn":
        return dict(w0=me + "0.weight", b0=me + "0.bias", w2=me + "2.weight", b2=me + "2.bias")
    return dict(win=me + "attn.in_proj_weight", bin=me + "attn.in_proj_bias", wo=me + "attn.out_proj.weight",
                bo=me + "attn.out_proj.bias", w1=me + "linear1.weight", b1=me + "linear1.bias",
                w2=me + "linear2.weight", b2=me + "linear2.bias")


UME = "flow_matching.meta_encoder."


def _unet_prep(u, P):
    """The step's GEMM weight layouts of the U-Net's convs (kdfm_convw_prep): downs (out, 4 in) tap-major, the
    bottleneck's forward and flipped data-gradient layouts, the transposed convs (in, out, 4) as (in, 4 out)."""
    for i in range(u.nl):
        K.convw_prep(P[UME + f"downs.{i}.weight"], fwd=u.wd[i])
    K.convw_prep(P[UME + "bottleneck.weight"], fwd=u.wbf, bwd=u.wbb)
    for j in range(u.nl):
        K.convw_prep(P[UME + f"ups.{j}.weight"], fwd=u.wu[j])


def _unet_fwd(u, P, k, x, out, R, rscale):
    """UNet1D on slab k's [x | e] rows (B * T, Ci) -> out = v (R None) or R + rscale * v (B * T, Cs)."""
    B, L, nl = u.B, u.L, u.nl
    inp = x
    for i in range(nl):   # Conv1d(k 4, s 2, p 1): unfold + GEMM, straight into the level's skip columns
        l = i + 1
        cols = u.cols[:B * L[l] * 4 * u.cin[i]].view(B * L[l], 4 * u.cin[i])
        K.unfold1d(inp, cols, B, L[i], L[l])
        skip = u.cat[l][k][:, u.cx[l]:]
        K.linear(cols, u.wd[i], P[UME + f"downs.{i}.bias"], skip)
        inp = skip
    # bottleneck Conv1d(k 3, p 1) into the deepest level's x part
    K.conv3(inp, u.wbf, P[UME + "bottleneck.bias"], u.cat[nl][k][:, :u.cx[nl]], L[nl])
    for j, (ci, co) in enumerate(u.ups):   # ConvTranspose1d(k 4, s 2, p 1) = GEMM + fold (zero pad past 2 L_l)
        l = nl - j
        Z = u.z[:B * L[l] * 4 * co].view(B * L[l], 4 * co)
        K.linear_dx(u.cat[l][k], u.wu[j], Z)
        dst, Lout = (u.cat[l - 1][k][:, :u.cx[l - 1]], L[l - 1]) if l > 1 else (u.up_last[k], 2 * L[1])
        K.fold1d(Z, dst, B, L[l], Lout, bias=P[UME + f"ups.{j}.bias"], Lvalid=2 * L[l])
    epi = _lib.EPI_RESID if R is not None else 0
    K.linear(u.up_last[k], P[UME + "final.weight"].view(out.shape[1], -1), P[UME + "final.bias"], out, epi=epi, R=R,
             rscale=rscale)


def _unet_bwd(u, P, G, k, x, dv, dembed):
    """dembed = d/d[x | e] of slab k's U-Net given dv; parameter gradients into G (final / biases directly, the
    conv weights into the GEMM-layout accumulators u.gd / u.gb / u.gu, re-laid out once in meta_backward)."""
    B, L, nl = u.B, u.L, u.nl
    Cs = dv.shape[1]
    K.linear_dw(dv, u.up_last[k], G[UME + "final.weight"].view(Cs, -1), db=G[UME + "final.bias"])
    K.linear_dx(dv, P[UME + "final.weight"].view(Cs, -1), u.dup)
    for j in range(nl - 1, -1, -1):   # ups, last first: d_out -> dZ (unfold of the conv's own 2 L_l rows)
        ci, co = u.ups[j]
        l = nl - j
        dout, Lout = (u.dcat[l - 1][:, :u.cx[l - 1]], L[l - 1]) if l > 1 else (u.dup, 2 * L[1])
        # bias gradient: the sum over the 2 L_l frames the transposed conv writes (not the zero pad)
        db = u.dbcols[:B * 2 * L[l] * co].view(B * 2 * L[l], co)
        K.unfold1d(dout, db, B, Lout, 2 * L[l], K=1, S=1, P=0, Lvalid=2 * L[l])
        K.colsum(db, G[UME + f"ups.{j}.bias"])
        dZ = u.cols[:B * L[l] * 4 * co].view(B * L[l], 4 * co)
        K.unfold1d(dout, dZ, B, Lout, L[l], Lvalid=2 * L[l])
        K.linear_dw(u.cat[l][k], dZ, u.gu[j])
        K.linear(dZ, u.wu[j], None, u.dcat[l])
    # bottleneck: its output gradient is the deepest level's x part; the input is that level's skip
    dy = u.dcat[nl][:, :u.cx[nl]]
    skip = u.cat[nl][k][:, u.cx[nl]:]
    K.conv3_dw(dy, skip, u.gb, L[nl], db=G[UME + "bottleneck.bias"])
    # the skip columns of dcat[l] accumulate the skip's whole gradient in place (the up path's share, then the
    # down path's: R aliases the output, each element read and written by one thread)
    dsk = u.dcat[nl][:, u.cx[nl]:]
    K.conv3(dy, u.wbb, None, dsk, L[nl], R=dsk, rscale=1.0)
    for i in range(nl - 1, -1, -1):   # downs, deepest first: dW from the re-unfolded input, data grad = GEMM + fold
        l = i + 1
        inp = x if i == 0 else u.cat[i][k][:, u.cx[i]:]
        cols = u.cols[:B * L[l] * 4 * u.cin[i]].view(B * L[l], 4 * u.cin[i])
        K.unfold1d(inp, cols, B, L[i], L[l])
        dy = u.dcat[l][:, u.cx[l]:]
        K.linear_dw(dy, cols, u.gd[i], db=G[UME + f"downs.{i}.bias"])
        K.linear_dx(dy, u.wd[i], cols)
        if i == 0:
            K.fold1d(cols, dembed, B, L[l], L[0])
        else:
            dprev = u.dcat[i][:, u.cx[i]:]
            K.fold1d(cols, dprev, B, L[l], L[i], R=dprev)


def _meta_fwd(ws, P, nm, k, out, R, rscale, seed=None, bn_running=None, train=True):
    """One meta-encoder evaluation on slab k: out = v (R None) or R + rscale * v."""
    Cs = out.shape[1]
    x = ws.embed[k]
    if ws.meta == "unet":
        _unet_fwd(ws.unet, P, k, x, out, R, rscale)
        return
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
    if ws.meta == "unet":
        _unet_bwd(ws.unet, P, G, k, x, dv, dembed)
        return
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
    if ws.meta == "unet":
        _unet_prep(ws.unet, P)
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
    if ws.meta == "unet":
        u = ws.unet
        _unet_prep(u, P)   # (the forward's layouts of the same weights: re-prepared, the step may reuse them)
        for g_ in u.gd + u.gu + [u.gb]:
            K.fill(g_, 0.0)
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
    if ws.meta == "unet":
        u = ws.unet
        for i in range(u.nl):
            K.convw_grad(u.gd[i], G[UME + f"downs.{i}.weight"])
            K.convw_grad(u.gu[i], G[UME + f"ups.{i}.weight"])
        K.convw_grad(u.gb, G[UME + "bottleneck.weight"])


__all__ = ["META_TYPES", "MetaFMWorkspace", "meta_forward", "meta_backward"]
