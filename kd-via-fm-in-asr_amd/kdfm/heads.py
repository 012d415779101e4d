"""ver5 KD heads, forward and backward, over ALL layers at once.

Reference: DistilFlowMatchingCTCModelBPE._compute_v_losses_one_layer, version 5
(asr_train_diffm.py:645-702) applied per layer pair in training_step (:773-792) with the shared
head modules TeacherAutoEncoder (:400-414), StudentProjector (:416-423), NoiseAdapter (:425-442),
SimpleDenoiser(steps=9) (:444-460) and FMLatent -> FlowMatchingModule (:462-497, :1270-1427;
meta_encoder 'mlp', shape_transform 'linear', rectified schedule :852-856).

Because the head modules are shared by the 16 layers, running them once over the stacked
(16*B*T') rows is exactly the reference's per-layer loop, and the per-layer MSE means summed over
layers equal one sum of squares over the stack divided by the per-layer element count.

Layout: channels-last rows (layer, utterance, frame); the time convolutions of the denoiser use the
CONV operand mode of the GEMM (rows grouped in utterances of T' frames, zero padding per utterance).
FM recurrence (rectified, s = steps): x_{j+1} = x_j - v_j / s with v_j = W2 relu(W1 [x_j; e(t_j)] + b1) + b2,
t_j = (s - j)/s; loss = mean((Wst (z_deno - v_{s-1}) + bst - z_t)^2).
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K
from .overlap import WGRAD
from .config import Ver5Config

SALT_HEADS = 7


def _empty(*shape, dev):
    return torch.empty(*shape, device=dev, dtype=torch.float32)


class HeadsWorkspace:
    """Per-step re-laid-out head weights (conv weights in GEMM layouts, FM per-step biases)."""

    def __init__(self, cfg: Ver5Config, dev):
        L, E, S = cfg.latent, cfg.time_embed_dim, cfg.fm_steps
        self.wconv = _empty(4, L, 3 * L, dev=dev)      # denoiser conv weights in GEMM layouts
        self.w1f, self.w1b, self.w2f, self.w2b = self.wconv.unbind(0)
        self.wconv_h = None
        if K.twins_enabled():
            self.wconv_h = torch.empty(4, L, 3 * L, device=dev, dtype=torch.bfloat16)
            K.register_bf16_twin(self.wconv, self.wconv_h)
        self.g1 = _empty(L, 3 * L, dev=dev)
        self.g2 = _empty(L, 3 * L, dev=dev)
        self.cvec = _empty(S, L, dev=dev)
        self.evec = _empty(S, E, dev=dev)
        self.dc = _empty(S, L, dev=dev)


def heads_forward(cfg: Ver5Config, P, s_feats, t_feats, T, ws: HeadsWorkspace, acc, *, seed, eps=None, save=True):
    """s_feats (n, 88) and t_feats (n, 176) stacked student/teacher layer outputs (n = layers*B*T).
    acc: device (2,) f32 accumulators [recon, fm] (added to).  Returns ctx for backward."""
    dev = s_feats.device
    n = s_feats.shape[0]
    Lt, Ct = cfg.latent, cfg.d_teacher
    B_eff = n // T   # layers * B
    n_layers = cfg.n_layers
    per_layer_rows = n // n_layers
    # ---- TeacherAutoEncoder + recon MSE (mean over B*C*T per layer, summed over layers) ----
    zt = _empty(n, Lt, dev=dev)
    K.linear(t_feats, P["tae.enc.weight"].view(Lt, Ct), P["tae.enc.bias"], zt)
    drec = _empty(n, Ct, dev=dev)
    inv_rec = 1.0 / (per_layer_rows * Ct)
    K.linear(zt, P["tae.dec.weight"].view(Ct, Lt), P["tae.dec.bias"], drec, R=t_feats, rscale=2.0 * inv_rec,
             mse=(acc[0:1], inv_rec))
    # ---- StudentProjector ----
    zs = _empty(n, Lt, dev=dev)
    K.linear(s_feats, P["sproj.proj.weight"].view(Lt, cfg.d_student), P["sproj.proj.bias"], zs)
    # ---- NoiseAdapter ----
    hA = _empty(n, Lt, dev=dev)
    K.linear(zs, P["adapter.gamma_head.0.weight"].view(Lt, Lt), P["adapter.gamma_head.0.bias"], hA,
             epi=_lib.EPI_RELU)
    zn = _empty(n, Lt, dev=dev)
    gamma = _empty(n, dev=dev)
    K.adapter_fwd(zs, hA, P["adapter.gamma_head.2.weight"].view(-1), P["adapter.gamma_head.2.bias"], eps, zn, gamma,
                  seed, SALT_HEADS)
    # ---- SimpleDenoiser: x <- x - net(x)/steps ----
    K.convw_prep(P["denoiser.net.0.weight"], fwd=ws.w1f, bwd=ws.w1b)
    K.convw_prep(P["denoiser.net.2.weight"], fwd=ws.w2f, bwd=ws.w2b)
    if K.get_math() == "bf16" and ws.wconv_h is not None:
        K.cast_bf16(ws.wconv, ws.wconv_h)
    ds = cfg.denoiser_steps
    xs = [zn]
    acts = []
    for _ in range(ds):
        a = _empty(n, Lt, dev=dev)
        K.conv3(xs[-1], ws.w1f, P["denoiser.net.0.bias"], a, T, epi=_lib.EPI_RELU, tag="deno_conv")
        xn = _empty(n, Lt, dev=dev)
        K.conv3(a, ws.w2f, P["denoiser.net.2.bias"], xn, T, R=xs[-1], rscale=-1.0 / ds, tag="deno_conv")
        acts.append(a)
        xs.append(xn)
    zd = xs[-1]
    # ---- FlowMatchingModule (mlp meta-encoder, linear shape transform, rectified) ----
    fm = "fm_latent.fm."
    S_ = cfg.fm_steps
    E = cfg.time_embed_dim
    W1 = P[fm + "meta_encoder.0.weight"]          # (L, L+E)
    W1x = W1[:, :Lt]
    W2 = P[fm + "meta_encoder.2.weight"]
    K.fm_step_bias(P[fm + "time_embed.weight"].view(-1), P[fm + "time_embed.bias"], W1, P[fm + "meta_encoder.0.bias"],
                   ws.cvec, ws.evec, Lt, E, S_)
    fx = [zd]
    fa = []
    v = None
    for j in range(S_):
        a = _empty(n, Lt, dev=dev)
        K.linear(fx[-1], W1x, ws.cvec[j], a, epi=_lib.EPI_RELU)
        fa.append(a)
        if j < S_ - 1:
            xn = _empty(n, Lt, dev=dev)
            K.linear(a, W2, P[fm + "meta_encoder.2.bias"], xn, epi=_lib.EPI_RESID, R=fx[-1], rscale=-1.0 / S_)
            fx.append(xn)
        else:
            v = _empty(n, Lt, dev=dev)
            K.linear(a, W2, P[fm + "meta_encoder.2.bias"], v)
    # noise_scheduled_x = (dalpha*s - v) / (-dsigma) = s - v   (rectified: dalpha = 1, dsigma = -1)
    nsx = _empty(n, Lt, dev=dev)
    K.axpby(zd, v, nsx, 1.0, -1.0)
    dtr = _empty(n, Lt, dev=dev)
    inv_fm = 1.0 / (per_layer_rows * Lt)
    K.linear(nsx, P[fm + "shape_transformation_function.weight"], P[fm + "shape_transformation_function.bias"], dtr,
             R=zt, rscale=2.0 * inv_fm, mse=(acc[1:2], inv_fm))
    if not save:
        return None
    return dict(n=n, T=T, zt=zt, drec=drec, zs=zs, hA=hA, gamma=gamma, eps=eps, xs=xs, acts=acts, fx=fx, fa=fa,
                nsx=nsx, dtr=dtr, s_feats=s_feats, t_feats=t_feats, B_eff=B_eff)


def heads_backward(cfg: Ver5Config, P, G, ctx, ws: HeadsWorkspace, ds_feats, *, seed):
    """Accumulates head parameter grads into G and writes d(loss)/d(student layer outputs) into
    ds_feats (n, 88)."""
    n, T = ctx["n"], ctx["T"]
    dev = ds_feats.device
    Lt, Ct = cfg.latent, cfg.d_teacher
    fm = "fm_latent.fm."
    S_ = cfg.fm_steps
    E = cfg.time_embed_dim
    W1 = P[fm + "meta_encoder.0.weight"]
    W1x = W1[:, :Lt]
    dW1 = G[fm + "meta_encoder.0.weight"]
    dW1x = dW1[:, :Lt]
    W2 = P[fm + "meta_encoder.2.weight"]
    # ---- FM loss: tr = Wst nsx + b ; d_tr given ----
    dtr = ctx["dtr"]
    WGRAD.run(lambda: K.linear_dw(dtr, ctx["nsx"], G[fm + "shape_transformation_function.weight"], db=G[fm + "shape_transformation_function.bias"]), dtr, ctx["nsx"])
    dnsx = _empty(n, Lt, dev=dev)
    K.linear_dx(dtr, P[fm + "shape_transformation_function.weight"], dnsx)
    # nsx = zd - v  ->  d zd += dnsx ; dv = -dnsx
    fx, fa = ctx["fx"], ctx["fa"]
    gx_next = None     # grad wrt fx[j+1]
    K.fill(ws.dc, 0.0)
    for j in range(S_ - 1, -1, -1):
        if j == S_ - 1:
            gsrc, alpha = dnsx, -1.0          # dv_{S-1} = -dnsx
        else:
            gsrc, alpha = gx_next, -1.0 / S_  # dv_j = -(1/S) g_{x_{j+1}}
        WGRAD.run(lambda: K.linear_dw(gsrc, fa[j], G[fm + "meta_encoder.2.weight"], alpha=alpha, db=G[fm + "meta_encoder.2.bias"]), gsrc, fa[j])
        da = _empty(n, Lt, dev=dev)
        K.linear_dx(gsrc, W2, da, epi=_lib.EPI_DRELU, aux=fa[j], alpha=alpha)
        WGRAD.run(lambda: K.linear_dw(da, fx[j], dW1x, db=ws.dc[j]), da, fx[j])
        gx = _empty(n, Lt, dev=dev)
        if gx_next is None:
            K.linear_dx(da, W1x, gx)
        else:
            K.linear_dx(da, W1x, gx, R=gx_next, rscale=1.0)
        gx_next = gx
        del da
    WGRAD.join()  # ws.dc (per-step bias grads) is produced on the side stream
    K.fm_time_bwd(ws.dc, ws.evec, W1, dW1, G[fm + "meta_encoder.0.bias"], G[fm + "time_embed.weight"].view(-1),
                  G[fm + "time_embed.bias"], Lt, E, S_)
    # d zd = gx_0 + dnsx
    g = _empty(n, Lt, dev=dev)
    K.axpby(gx_next, dnsx, g, 1.0, 1.0)
    del gx_next, dnsx
    # ---- denoiser backward ----
    ds = cfg.denoiser_steps
    xs, acts = ctx["xs"], ctx["acts"]
    K.fill(ws.g1, 0.0)
    K.fill(ws.g2, 0.0)
    for i in range(ds - 1, -1, -1):
        # x_{i+1} = x_i - (1/ds)(conv(a_i, W2) + b2)
        WGRAD.run(lambda: K.conv3_dw(g, acts[i], ws.g2, T, alpha=-1.0 / ds, db=G["denoiser.net.2.bias"]), g, acts[i])
        da = _empty(n, Lt, dev=dev)
        K.conv3(g, ws.w2b, None, da, T, epi=_lib.EPI_DRELU, aux=acts[i], alpha=-1.0 / ds, tag="deno_conv")
        WGRAD.run(lambda: K.conv3_dw(da, xs[i], ws.g1, T, db=G["denoiser.net.0.bias"]), da, xs[i])
        gi = _empty(n, Lt, dev=dev)
        K.conv3(da, ws.w1b, None, gi, T, R=g, rscale=1.0, tag="deno_conv")
        g = gi
        del da
    WGRAD.join()  # ws.g1 / ws.g2 are produced on the side stream
    K.convw_grad(ws.g1, G["denoiser.net.0.weight"])
    K.convw_grad(ws.g2, G["denoiser.net.2.weight"])
    # ---- NoiseAdapter backward ----
    zs, hA = ctx["zs"], ctx["hA"]
    dzs_direct = _empty(n, Lt, dev=dev)
    dh = _empty(n, Lt, dev=dev)
    K.adapter_bwd(g, zs, hA, ctx["gamma"], P["adapter.gamma_head.2.weight"].view(-1), ctx["eps"], dzs_direct, dh,
                  G["adapter.gamma_head.2.weight"].view(-1), G["adapter.gamma_head.2.bias"], seed, SALT_HEADS)
    del g
    WGRAD.run(lambda: K.linear_dw(dh, zs, G["adapter.gamma_head.0.weight"].view(Lt, Lt), db=G["adapter.gamma_head.0.bias"]), dh, zs)
    dzs = _empty(n, Lt, dev=dev)
    K.linear_dx(dh, P["adapter.gamma_head.0.weight"].view(Lt, Lt), dzs, R=dzs_direct, rscale=1.0)
    del dh, dzs_direct
    # ---- StudentProjector backward -> grads wrt the student layer outputs ----
    WGRAD.run(lambda: K.linear_dw(dzs, ctx["s_feats"], G["sproj.proj.weight"].view(Lt, cfg.d_student), db=G["sproj.proj.bias"]), dzs, ctx["s_feats"])
    K.linear_dx(dzs, P["sproj.proj.weight"].view(Lt, cfg.d_student), ds_feats)
    del dzs
    # ---- TeacherAutoEncoder backward (recon only; z_t is detached for the FM target) ----
    drec, zt = ctx["drec"], ctx["zt"]
    WGRAD.run(lambda: K.linear_dw(drec, zt, G["tae.dec.weight"].view(Ct, Lt), db=G["tae.dec.bias"]), drec, zt)
    dzt = _empty(n, Lt, dev=dev)
    K.linear_dx(drec, P["tae.dec.weight"].view(Ct, Lt), dzt)
    WGRAD.run(lambda: K.linear_dw(dzt, ctx["t_feats"], G["tae.enc.weight"].view(Lt, Ct), db=G["tae.enc.bias"]), dzt, ctx["t_feats"])
    