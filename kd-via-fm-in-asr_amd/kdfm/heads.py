"""KD heads of every model version (ver1-ver8), forward and backward, over ALL layers at once.

Reference: DistilFlowMatchingCTCModelBPE._compute_v_losses_one_layer (asr_train_diffm.py:645-729)
applied per layer pair in training_step (:773-792) with the shared head modules TeacherAutoEncoder
(:400-414), StudentProjector (:416-423), NoiseAdapter (:425-442), SimpleDenoiser(steps=9)
(:444-460) and FMLatent -> FlowMatchingModule (:462-497, :1270-1427; meta_encoder 'mlp',
shape_transform 'linear', rectified schedule :852-856).  Per version (z_s = sproj(s), z_t = the
detached teacher latent, kd = MSE or L1 by kd_loss_type):
  1 kd_pre = kd(z_s)                 5 fm_post = FM(deno(adapt(z_s)))
  2 fm_pre = FM(z_s)                 6 fm_pre, x = FM(z_s); fm_post = FM2(deno(adapt(x)))
  3 kd_post = kd(deno(adapt(z_s)))   7 fm_pre = FM(z_s); fm_post = FM2(deno(adapt(z_s)))
  4 fm_pre = FM(z_s); kd_post = kd(deno(adapt(z_s)))    8 fm_pre, x = FM(z_s); kd_post = kd(deno(adapt(x)))
with the teacher auto-encoder's recon MSE always on.

Because the head modules are shared by the 16 layers, running them once over the stacked
(16*B*T') rows is exactly the reference's per-layer loop, and the per-layer means summed over
layers equal one sum over the stack divided by the per-layer element count.

Layout: channels-last rows (layer, utterance, frame); the time convolutions of the denoiser use the
CONV operand mode of the GEMM (rows grouped in utterances of T' frames, zero padding per utterance).
FM recurrence (rectified, s = steps): x_{j+1} = x_j - v_j / s with v_j = W2 relu(W1 [x_j; e(t_j)] + b1) + b2,
t_j = (s - j)/s; loss = mean((Wst (x_0 - v_{s-1}) + bst - z_t)^2); the module's second output is x_s.
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K
from .overlap import WGRAD
from .config import Ver5Config

SALT_HEADS = 7
# loss slots of the accumulator heads_forward adds into
RECON, KD_PRE, FM_PRE, KD_POST, FM_POST = range(5)


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
        # the DiffKD denoiser's own GEMM-layout weights and weight-gradient accumulators (its backward
        # can overlap the version denoiser's on the weight-gradient stream)
        self.dk_wconv = _empty(4, L, 3 * L, dev=dev)
        self.dk_g1 = _empty(L, 3 * L, dev=dev)
        self.dk_g2 = _empty(L, 3 * L, dev=dev)
        # per FM module: per-step first-layer bias (time embedding folded in), time features, bias grads
        self.fm = {}
        for pre in ("fm_latent.fm.", "fm_latent_2.fm."):
            self.fm[pre] = (_empty(S, L, dev=dev), _empty(S, E, dev=dev), _empty(S, L, dev=dev))
        self.cvec, self.evec, self.dc = self.fm["fm_latent.fm."]
        # NoiseAdapter gamma-head output-layer gradient [dw2 (L) | db2] of one heads call, folded into G on
        # the weight-gradient stream (two layer halves run their backward concurrently: a direct
        # read-modify-write of G from both issuing streams could lose one half's sum)
        self.adw = _empty(1, L + 1, dev=dev)


# ------------------------------------------------------------------------------------------------
# building blocks
# ------------------------------------------------------------------------------------------------

def _kd(cfg, a, b, slot, inv, dev):
    """kd_crit(a, b) (nn.MSELoss / nn.L1Loss, mean) added into slot; returns d(loss)/da (elementwise,
    computed in the same pass)."""
    g = _empty(*a.shape, dev=dev)
    if cfg.kd_loss_type == "l1":
        K.l1(a, b, slot, inv, grad=g, gscale=inv)
    else:
        K.mse(a, b, slot, inv, grad=g, gscale=2.0 * inv)
    return g


def _fm_fused(Lt):
    """bf16 math runs the fused chain kernels (csrc/fmchain.hip); the f32 parity mode keeps the
    per-step GEMMs (KDFM_FM_FUSED=0 forces them in bf16 too)."""
    return K.get_math() == "bf16" and Lt == 96 and _FM_FUSED


_FM_FUSED = __import__("os").environ.get("KDFM_FM_FUSED", "1") == "1"


def _fm_forward(cfg, P, pre, ws, x0, zt, slot, inv, need_out, dev):
    """FlowMatchingModule over rows x0 (n, L) against z_t: loss into slot; ctx for backward.  With
    need_out the module's second output x_s is materialised (versions 6 and 8 feed it onward)."""
    n, Lt = x0.shape
    S_ = cfg.fm_steps
    E = cfg.time_embed_dim
    W1 = P[pre + "meta_encoder.0.weight"]          # (L, L+E)
    W1x = W1[:, :Lt]
    W2 = P[pre + "meta_encoder.2.weight"]
    cvec, evec, _ = ws.fm[pre]
    K.fm_step_bias(P[pre + "time_embed.weight"].view(-1), P[pre + "time_embed.bias"], W1, P[pre + "meta_encoder.0.bias"],
                   cvec, evec, Lt, E, S_)
    if _fm_fused(Lt):
        X = torch.empty(S_, n, Lt, device=dev, dtype=torch.bfloat16)
        A = torch.empty(S_, n, Lt, device=dev, dtype=torch.bfloat16)
        nsx = _empty(n, Lt, dev=dev)
        dtr = _empty(n, Lt, dev=dev)
        xs = _empty(n, Lt, dev=dev) if need_out else None
        with K.span("fm_chain_fwd"):
            K.fm_chain_fwd(x0, zt, W1, cvec, W2, P[pre + "meta_encoder.2.bias"],
                           P[pre + "shape_transformation_function.weight"],
                           P[pre + "shape_transformation_function.bias"], X, A, nsx, dtr, xs, slot, inv, S_)
        return dict(pre=pre, fused=True, X=X, A=A, nsx=nsx, dtr=dtr), xs
    fx = [x0]
    fa = []
    v = None
    for j in range(S_):
        a = _empty(n, Lt, dev=dev)
        K.linear(fx[-1], W1x, cvec[j], a, epi=_lib.EPI_RELU, tag="fm_up")
        fa.append(a)
        if j < S_ - 1:
            xn = _empty(n, Lt, dev=dev)
            K.linear(a, W2, P[pre + "meta_encoder.2.bias"], xn, epi=_lib.EPI_RESID, R=fx[-1], rscale=-1.0 / S_,
                     tag="fm_down")
            fx.append(xn)
        else:
            v = _empty(n, Lt, dev=dev)
            K.linear(a, W2, P[pre + "meta_encoder.2.bias"], v, tag="fm_down")
    xs = None
    if need_out:
        xs = _empty(n, Lt, dev=dev)
        K.axpby(fx[-1], v, xs, 1.0, -1.0 / S_)
    # noise_scheduled_x = (dalpha*s - v) / (-dsigma) = s - v   (rectified: dalpha = 1, dsigma = -1)
    nsx = _empty(n, Lt, dev=dev)
    K.axpby(x0, v, nsx, 1.0, -1.0)
    dtr = _empty(n, Lt, dev=dev)
    K.linear(nsx, P[pre + "shape_transformation_function.weight"], P[pre + "shape_transformation_function.bias"], dtr,
             R=zt, rscale=2.0 * inv, mse=(slot, inv))
    return dict(pre=pre, fx=fx, fa=fa, nsx=nsx, dtr=dtr), xs


def _fm_backward(cfg, P, G, ws, c, gxs, dev):
    """Backward of _fm_forward: parameter grads into G; returns d/d x0.  gxs: optional gradient
    wrt the module's x_s output."""
    pre = c["pre"]
    n, Lt = c["dtr"].shape
    S_ = cfg.fm_steps
    E = cfg.time_embed_dim
    W1 = P[pre + "meta_encoder.0.weight"]
    W1x = W1[:, :Lt]
    dW1 = G[pre + "meta_encoder.0.weight"]
    dW1x = dW1[:, :Lt]
    W2 = P[pre + "meta_encoder.2.weight"]
    _, evec, dc = ws.fm[pre]
    dtr, nsx = c["dtr"], c["nsx"]
    WGRAD.run(lambda: K.linear_dw(dtr, nsx, G[pre + "shape_transformation_function.weight"],
                                  db=G[pre + "shape_transformation_function.bias"]), dtr, nsx)
    if c.get("fused"):
        X, A = c["X"], c["A"]
        DV = torch.empty_like(A)
        DA = torch.empty_like(A)
        g = _empty(n, Lt, dev=dev)
        with K.span("fm_chain_bwd"):
            K.fm_chain_bwd(dtr, A, gxs, W1, W2, P[pre + "shape_transformation_function.weight"], DV, DA, g, S_)
        # weight gradients from the saved bf16 operands: dW2 over all steps' rows at once, dW1x (and
        # the per-step first-layer bias grads dc_j) per step
        K.fill(dc, 0.0)
        WGRAD.run(lambda: K.wgrad_bf16(DV.view(S_ * n, Lt), A.view(S_ * n, Lt), G[pre + "meta_encoder.2.weight"],
                                       db=G[pre + "meta_encoder.2.bias"]), DV, A)
        # dW1x over all S_ steps' rows in one launch, with the per-step bias grads dc_j as segment
        # columns (kdfm_wgrad_bf16_seg; was S_ launches + S_ folds)
        if K.wgrad_bf16_seg_ok(S_ * n, Lt, Lt, n):
            WGRAD.run(lambda: K.wgrad_bf16_seg(DA.view(S_ * n, Lt), X.view(S_ * n, Lt), dW1x, dc, n), DA, X)
        else:
            for j in range(S_):
                WGRAD.run(lambda j=j: K.wgrad_bf16(DA[j], X[j], dW1x, db=dc[j]), DA, X)
        # dc is produced on the side stream: fold it there too (no main-stream join); a deferred fold of the
        # products writing it completes first
        def time_bwd():
            K.wgrad_fold_flush()
            K.fm_time_bwd(dc, evec, W1, dW1, G[pre + "meta_encoder.0.bias"], G[pre + "time_embed.weight"].view(-1),
                          G[pre + "time_embed.bias"], Lt, E, S_)
        WGRAD.run(time_bwd)
        return g
    fx, fa = c["fx"], c["fa"]
    dnsx = _empty(n, Lt, dev=dev)
    K.linear_dx(dtr, P[pre + "shape_transformation_function.weight"], dnsx)
    # nsx = x0 - v_{S-1}  ->  d x0 += dnsx ; dv_{S-1} = -dnsx (- gxs / S when x_S is used)
    last, last_alpha = dnsx, -1.0
    if gxs is not None:
        last = _empty(n, Lt, dev=dev)
        K.axpby(dnsx, gxs, last, -1.0, -1.0 / S_)
        last_alpha = 1.0
    gx_next = gxs     # grad wrt fx[j+1] (x_S for the last step)
    K.fill(dc, 0.0)
    for j in range(S_ - 1, -1, -1):
        if j == S_ - 1:
            gsrc, alpha = last, last_alpha
        else:
            gsrc, alpha = gx_next, -1.0 / S_  # dv_j = -(1/S) g_{x_{j+1}}
        WGRAD.run(lambda gsrc=gsrc, alpha=alpha, j=j: K.linear_dw(gsrc, fa[j], G[pre + "meta_encoder.2.weight"],
                                                                  alpha=alpha, db=G[pre + "meta_encoder.2.bias"]),
                  gsrc, fa[j])
        da = _empty(n, Lt, dev=dev)
        K.linear_dx(gsrc, W2, da, epi=_lib.EPI_DRELU, aux=fa[j], alpha=alpha)
        WGRAD.run(lambda da=da, j=j: K.linear_dw(da, fx[j], dW1x, db=dc[j]), da, fx[j])
        gx = _empty(n, Lt, dev=dev)
        if gx_next is None:
            K.linear_dx(da, W1x, gx)
        else:
            K.linear_dx(da, W1x, gx, R=gx_next, rscale=1.0)
        gx_next = gx
        del da
    # dc (per-step bias grads) is produced on the side stream: fold it there too
    WGRAD.run(lambda: K.fm_time_bwd(dc, evec, W1, dW1, G[pre + "meta_encoder.0.bias"],
                                    G[pre + "time_embed.weight"].view(-1), G[pre + "time_embed.bias"], Lt, E, S_))
    g = _empty(n, Lt, dev=dev)
    K.axpby(gx_next, dnsx, g, 1.0, 1.0)
    return g


_DENO_FUSED = __import__("os").environ.get("KDFM_DENOISE_FUSED", "1") == "1"


def _deno_fused(Lt):
    """bf16 math runs the fused SimpleDenoiser chain kernels (csrc/denoise.hip); the f32 parity mode
    keeps the per-step conv GEMMs (KDFM_DENOISE_FUSED=0 forces them in bf16 too)."""
    return K.get_math() == "bf16" and Lt == 96 and _DENO_FUSED


class _Deno:
    """Weight names and workspace slots of one SimpleDenoiser-shaped chain: the version's denoiser
    (asr_train_diffm.py:444-460, `denoiser.net.{0,2}`) or DiffKD's (:350-354, `diffkd.denoiser.{0,2}`)."""

    def __init__(self, ws, pre, steps, diffkd=False):
        self.w1, self.w2 = pre + "0.weight", pre + "2.weight"
        self.b1, self.b2 = pre + "0.bias", pre + "2.bias"
        self.steps = steps
        if diffkd:
            self.wconv, self.wconv_h, self.g1, self.g2 = ws.dk_wconv, None, ws.dk_g1, ws.dk_g2
        else:
            self.wconv, self.wconv_h, self.g1, self.g2 = ws.wconv, ws.wconv_h, ws.g1, ws.g2
        self.w1f, self.w1b, self.w2f, self.w2b = self.wconv.unbind(0)


def _denoise_forward(P, dn: _Deno, zn, T, dev):
    """x <- x - net(x)/steps, `steps` times over rows zn; returns (ctx, x_steps)."""
    n, Lt = zn.shape
    ds = dn.steps
    if _deno_fused(Lt):
        X = torch.empty(ds, n, Lt, device=dev, dtype=torch.bfloat16)
        A = torch.empty(ds, n, Lt, device=dev, dtype=torch.bfloat16)
        out = _empty(n, Lt, dev=dev)
        with K.span("denoise_chain_fwd"):
            K.denoise_chain_fwd(zn, P[dn.w1], P[dn.b1], P[dn.w2], P[dn.b2], X, A, out, T, ds)
        return dict(fused=True, X=X, A=A), out
    K.convw_prep(P[dn.w1], fwd=dn.w1f, bwd=dn.w1b)
    K.convw_prep(P[dn.w2], fwd=dn.w2f, bwd=dn.w2b)
    if K.get_math() == "bf16" and dn.wconv_h is not None:
        K.cast_bf16(dn.wconv, dn.wconv_h)
    xs = [zn]
    acts = []
    for _ in range(ds):
        a = _empty(n, Lt, dev=dev)
        K.conv3(xs[-1], dn.w1f, P[dn.b1], a, T, epi=_lib.EPI_RELU, tag="deno_conv")
        xn = _empty(n, Lt, dev=dev)
        K.conv3(a, dn.w2f, P[dn.b2], xn, T, R=xs[-1], rscale=-1.0 / ds, tag="deno_conv")
        acts.append(a)
        xs.append(xn)
    return dict(xs=xs, acts=acts), xs[-1]


def _denoise_backward(P, G, dn: _Deno, c, g, T, dev):
    """g = d/d x_steps -> returns d/d x_0; parameter gradients into G (weight-gradient stream)."""
    n, Lt = g.shape
    ds = dn.steps
    if not c.get("fused"):
        return _denoise_backward_unfused(P, G, dn, c, g, T, dev)
    X, A = c["X"], c["A"]
    GV = torch.empty(ds, n, Lt, device=dev, dtype=torch.bfloat16)
    DA = torch.empty(ds, n, Lt, device=dev, dtype=torch.bfloat16)
    gin = _empty(n, Lt, dev=dev)
    with K.span("denoise_chain_bwd"):
        K.denoise_chain_bwd(g, A, P[dn.w1], P[dn.w2], GV, DA, gin, T, ds)

    def wgrads():
        # one row-parallel launch per conv over all ds steps (the stacked saves keep whole utterances)
        K.fill(dn.g1, 0.0)
        K.fill(dn.g2, 0.0)
        K.wgrad_bf16_conv(DA.view(ds * n, Lt), X.view(ds * n, Lt), dn.g1, T, db=G[dn.b1])
        K.wgrad_bf16_conv(GV.view(ds * n, Lt), A.view(ds * n, Lt), dn.g2, T, alpha=-1.0 / ds, db=G[dn.b2])
        K.wgrad_fold_flush()   # g1 / g2 are read below (deferred folds, conformer.fold_arena)
        K.convw_grad(dn.g1, G[dn.w1])
        K.convw_grad(dn.g2, G[dn.w2])
    WGRAD.run(wgrads, X, A, GV, DA)
    return gin


def _adapt_denoise_forward(cfg, P, ws, x, T, seed, eps, dev, salt=SALT_HEADS):
    """NoiseAdapter then the 9-step SimpleDenoiser over rows x; returns (ctx, z_deno).  salt: the counter-RNG
    stream of the adapter noise (one per layer-half call, so the halves draw independent noise)."""
    n, Lt = x.shape
    hA = _empty(n, Lt, dev=dev)
    K.linear(x, P["adapter.gamma_head.0.weight"].view(Lt, Lt), P["adapter.gamma_head.0.bias"], hA, epi=_lib.EPI_RELU)
    zn = _empty(n, Lt, dev=dev)
    gamma = _empty(n, dev=dev)
    K.adapter_fwd(x, hA, P["adapter.gamma_head.2.weight"].view(-1), P["adapter.gamma_head.2.bias"], eps, zn, gamma,
                  seed, salt)
    dctx, out = _denoise_forward(P, _Deno(ws, "denoiser.net.", cfg.denoiser_steps), zn, T, dev)
    dctx.update(x=x, hA=hA, gamma=gamma, eps=eps, salt=salt)
    return dctx, out


def _adapt_denoise_backward(cfg, P, G, ws, c, g, T, seed, dev):
    """g = d/d z_deno -> returns d/d (adapter input)."""
    n, Lt = g.shape
    g = _denoise_backward(P, G, _Deno(ws, "denoiser.net.", cfg.denoiser_steps), c, g, T, dev)
    x, hA = c["x"], c["hA"]
    dx_direct = _empty(n, Lt, dev=dev)
    dh = _empty(n, Lt, dev=dev)
    adw = ws.adw
    K.fill(adw, 0.0)
    K.adapter_bwd(g, x, hA, c["gamma"], P["adapter.gamma_head.2.weight"].view(-1), c["eps"], dx_direct, dh,
                  adw[0, :Lt], adw[0, Lt:], seed, c["salt"])
    del g
    gw2 = G["adapter.gamma_head.2.weight"].view(1, Lt)
    gb2 = G["adapter.gamma_head.2.bias"].view(1, 1)
    WGRAD.run(lambda: (K.axpby(adw[:, :Lt], gw2, gw2, 1.0, 1.0), K.axpby(adw[:, Lt:], gb2, gb2, 1.0, 1.0)), adw)
    WGRAD.run(lambda: K.linear_dw(dh, x, G["adapter.gamma_head.0.weight"].view(Lt, Lt),
                                  db=G["adapter.gamma_head.0.bias"]), dh, x)
    dx = _empty(n, Lt, dev=dev)
    K.linear_dx(dh, P["adapter.gamma_head.0.weight"].view(Lt, Lt), dx, R=dx_direct, rscale=1.0)
    return dx


def _denoise_backward_unfused(P, G, dn: _Deno, c, g, T, dev):
    """Per-step conv GEMMs of the denoiser backward (f32 parity mode); returns d/d(denoiser input)."""
    n, Lt = g.shape
    ds = dn.steps
    xs, acts = c["xs"], c["acts"]
    # the accumulators are zeroed on the weight-gradient stream, where they are accumulated and read
    WGRAD.run(lambda: (K.fill(dn.g1, 0.0), K.fill(dn.g2, 0.0)))
    for i in range(ds - 1, -1, -1):
        # x_{i+1} = x_i - (1/ds)(conv(a_i, W2) + b2)
        WGRAD.run(lambda g=g, i=i: K.conv3_dw(g, acts[i], dn.g2, T, alpha=-1.0 / ds, db=G[dn.b2]), g, acts[i])
        da = _empty(n, Lt, dev=dev)
        K.conv3(g, dn.w2b, None, da, T, epi=_lib.EPI_DRELU, aux=acts[i], alpha=-1.0 / ds, tag="deno_conv")
        WGRAD.run(lambda da=da, i=i: K.conv3_dw(da, xs[i], dn.g1, T, db=G[dn.b1]), da, xs[i])
        gi = _empty(n, Lt, dev=dev)
        K.conv3(da, dn.w1b, None, gi, T, R=g, rscale=1.0, tag="deno_conv")
        g = gi
        del da
    # the accumulators are produced on the side stream: re-lay them out there too
    WGRAD.run(lambda: (K.convw_grad(dn.g1, G[dn.w1]), K.convw_grad(dn.g2, G[dn.w2])))
    return g


# ------------------------------------------------------------------------------------------------
# the version graph
# ------------------------------------------------------------------------------------------------

def _diffkd_forward(cfg, P, Pfix, s_feats, t_feats, T, ws, acc, dev, layers=None):
    """DiffKDModule over every layer pair at once (asr_train_diffm.py:364-394), the layer mean of
    :795-800 folded into the MSE scales: z_t = encoder(t) (no gradient reaches the encoder, :382),
    ae = MSE(decoder(z_t), t), x = denoise^S(proj(s)), distill = MSE(x, z_t); acc += (ae + distill) / L."""
    n = s_feats.shape[0]
    Lt, Ct, Cs = cfg.latent, cfg.d_teacher, cfg.d_student
    rows = n // (layers or cfg.n_layers)
    zt = _empty(n, Lt, dev=dev)
    K.linear(t_feats, Pfix["diffkd.encoder.weight"].view(Lt, Ct), Pfix["diffkd.encoder.bias"], zt)
    drec = _empty(n, Ct, dev=dev)
    inv_rec = 1.0 / (rows * Ct * cfg.n_layers)
    K.linear(zt, P["diffkd.decoder.weight"].view(Ct, Lt), P["diffkd.decoder.bias"], drec, R=t_feats,
             rscale=2.0 * inv_rec, mse=(acc, inv_rec))
    zs = _empty(n, Lt, dev=dev)
    K.linear(s_feats, P["diffkd.proj.weight"].view(Lt, Cs), P["diffkd.proj.bias"], zs)
    dn = _Deno(ws, "diffkd.denoiser.", cfg.diffkd_steps, diffkd=True)
    dctx, zd = _denoise_forward(P, dn, zs, T, dev)
    inv = 1.0 / (rows * Lt * cfg.n_layers)
    gzd = _empty(n, Lt, dev=dev)
    K.mse(zd, zt, acc, inv, grad=gzd, gscale=2.0 * inv)
    return dict(zt=zt, drec=drec, dctx=dctx, gzd=gzd)


def _diffkd_backward(cfg, P, G, c, s_feats, T, ws, ds_feats, dev):
    """Backward of _diffkd_forward: decoder / proj / denoiser gradients into G, d/d(student layer
    outputs) ADDED into ds_feats."""
    Lt, Cs = cfg.latent, cfg.d_student
    Ct = cfg.d_teacher
    drec, zt = c["drec"], c["zt"]
    WGRAD.run(lambda: K.linear_dw(drec, zt, G["diffkd.decoder.weight"].view(Ct, Lt), db=G["diffkd.decoder.bias"]),
              drec, zt)
    dn = _Deno(ws, "diffkd.denoiser.", cfg.diffkd_steps, diffkd=True)
    dzs = _denoise_backward(P, G, dn, c["dctx"], c["gzd"], T, dev)
    WGRAD.run(lambda: K.linear_dw(dzs, s_feats, G["diffkd.proj.weight"].view(Lt, Cs), db=G["diffkd.proj.bias"]),
              dzs, s_feats)
    K.linear_dx(dzs, P["diffkd.proj.weight"].view(Lt, Cs), ds_feats, R=ds_feats, rscale=1.0)


def tae_forward(cfg: Ver5Config, P, t_feats, zt, drec, acc_recon, layers=None):
    """TeacherAutoEncoder over the stacked teacher layer outputs t_feats (n, d_teacher): z_t = enc(t) into
    zt (n, latent), the recon MSE (mean over B*C*T per layer, summed over layers) added into acc_recon and
    its gradient d/d t_rec into drec (n, d_teacher).  It reads nothing of the student, so the engine issues
    it on the teacher stream right after the teacher encoder (off the student's critical path)."""
    n = t_feats.shape[0]
    Lt, Ct = cfg.latent, cfg.d_teacher
    inv_rec = 1.0 / ((n // (layers or cfg.n_layers)) * Ct)
    K.linear(t_feats, P["tae.enc.weight"].view(Lt, Ct), P["tae.enc.bias"], zt)
    K.linear(zt, P["tae.dec.weight"].view(Ct, Lt), P["tae.dec.bias"], drec, R=t_feats, rscale=2.0 * inv_rec,
             mse=(acc_recon, inv_rec))


def tae_backward(cfg: Ver5Config, P, G, zt, drec, t_feats, dzt):
    """TeacherAutoEncoder backward (recon only; z_t is detached for every KD target): weight gradients
    only, nothing flows to the student, so all of it (the dz_t product included, into the caller's dzt)
    runs on the weight-gradient stream."""
    Lt, Ct = cfg.latent, cfg.d_teacher

    def work():
        K.linear_dw(drec, zt, G["tae.dec.weight"].view(Ct, Lt), db=G["tae.dec.bias"])
        K.linear_dx(drec, P["tae.dec.weight"].view(Ct, Lt), dzt)
        K.linear_dw(dzt, t_feats, G["tae.enc.weight"].view(Lt, Ct), db=G["tae.enc.bias"])
    WGRAD.run(work, drec, zt, t_feats, dzt)


def heads_forward(cfg: Ver5Config, P, s_feats, t_feats, T, ws: HeadsWorkspace, acc, *, seed, eps=None, save=True,
                  Pfix=None, acc_diffkd=None, tae=None, layers=None, salt=SALT_HEADS):
    """s_feats (n, d_student) and t_feats (n, d_teacher) stacked student/teacher layer outputs
    (n = layers*B*T').  acc: device (5,) f32 accumulators [recon, kd_pre, fm_pre, kd_post, fm_post]
    (added to; the slots a version does not use stay untouched).  tae: (zt, drec) when the caller has
    already run tae_forward (recon added into acc[0] there).  layers: how many hooked layers the rows
    stack (default all: the per-layer means; the engine runs the heads in two layer halves), salt: the
    adapter noise stream.  Returns ctx for backward."""
    dev = s_feats.device
    n = s_feats.shape[0]
    Lt, Ct = cfg.latent, cfg.d_teacher
    v = cfg.version
    per_layer_rows = n // (layers or cfg.n_layers)
    inv_lat = 1.0 / (per_layer_rows * Lt)
    # ---- TeacherAutoEncoder + recon MSE (mean over B*C*T per layer, summed over layers) ----
    if tae is None:
        zt, drec = _empty(n, Lt, dev=dev), _empty(n, Ct, dev=dev)
        tae_forward(cfg, P, t_feats, zt, drec, acc[RECON:RECON + 1], layers)
    else:
        zt, drec = tae
    # ---- StudentProjector ----
    zs = _empty(n, Lt, dev=dev)
    K.linear(s_feats, P["sproj.proj.weight"].view(Lt, cfg.d_student), P["sproj.proj.bias"], zs)
    ctx = dict(n=n, T=T, zt=zt, drec=drec, zs=zs, s_feats=s_feats, t_feats=t_feats)
    x_adapt = zs
    if v in (2, 4, 6, 7, 8):   # FM on the projected student latent
        ctx["fm_pre"], xs_out = _fm_forward(cfg, P, "fm_latent.fm.", ws, zs, zt, acc[FM_PRE:FM_PRE + 1], inv_lat,
                                            v in (6, 8), dev)
        if v in (6, 8):
            x_adapt = xs_out
    if v == 1:
        ctx["dkd_pre"] = _kd(cfg, zs, zt, acc[KD_PRE:KD_PRE + 1], inv_lat, dev)
    if v >= 3:
        ctx["ad"], zd = _adapt_denoise_forward(cfg, P, ws, x_adapt, T, seed, eps, dev, salt)
        if v in (3, 4, 8):
            ctx["dkd_post"] = _kd(cfg, zd, zt, acc[KD_POST:KD_POST + 1], inv_lat, dev)
        else:
            pre = "fm_latent.fm." if v == 5 else "fm_latent_2.fm."
            ctx["fm_post"], _ = _fm_forward(cfg, P, pre, ws, zd, zt, acc[FM_POST:FM_POST + 1], inv_lat, False, dev)
    if cfg.use_diffkd:
        ctx["diffkd"] = _diffkd_forward(cfg, P, Pfix, s_feats, t_feats, T, ws, acc_diffkd, dev, layers)
    return ctx if save else None


def heads_backward(cfg: Ver5Config, P, G, ctx, ws: HeadsWorkspace, ds_feats, *, seed):
    """Accumulates head parameter grads into G and writes d(loss)/d(student layer outputs) into
    ds_feats (n, d_student)."""
    n, T = ctx["n"], ctx["T"]
    dev = ds_feats.device
    Lt, Ct = cfg.latent, cfg.d_teacher
    v = cfg.version
    dzs = None
    gx_out = None     # gradient wrt the pre-FM's x_S (versions 6, 8)
    if v >= 3:
        if v in (3, 4, 8):
            gzd = ctx.pop("dkd_post")
        else:
            gzd = _fm_backward(cfg, P, G, ws, ctx.pop("fm_post"), None, dev)
        gx = _adapt_denoise_backward(cfg, P, G, ws, ctx.pop("ad"), gzd, T, seed, dev)
        del gzd
        if v in (6, 8):
            gx_out = gx
        else:
            dzs = gx
    if "fm_pre" in ctx:
        g = _fm_backward(cfg, P, G, ws, ctx.pop("fm_pre"), gx_out, dev)
        if dzs is None:
            dzs = g
        else:
            K.axpby(dzs, g, dzs, 1.0, 1.0)
    if v == 1:
        dzs = ctx.pop("dkd_pre")
    # ---- StudentProjector backward -> grads wrt the student layer outputs ----
    WGRAD.run(lambda: K.linear_dw(dzs, ctx["s_feats"], G["sproj.proj.weight"].view(Lt, cfg.d_student),
                                  db=G["sproj.proj.bias"]), dzs, ctx["s_feats"])
    K.linear_dx(dzs, P["sproj.proj.weight"].view(Lt, cfg.d_student), ds_feats)
    del dzs
    # ---- TeacherAutoEncoder backward ----
    tae_backward(cfg, P, G, ctx["zt"], ctx["drec"], ctx["t_feats"], _empty(n, Lt, dev=dev))
    if "diffkd" in ctx:
        _diffkd_backward(cfg, P, G, ctx.pop("diffkd"), ctx["s_feats"], T, ws, ds_feats, dev)
