"""Encoder-level flow matching with the dynamic step router on the engine.

Reference: asr_train.py's DistilFlowMatchingCTCModelBPE with use_flow_matching=True (the model family
before the latent heads of asr_train_diffm.py): for every hooked Conformer layer, a DynamicStepRouter
(:1021-1218) picks flow step counts from the time means of the student and teacher features and a
layer embedding, a strategy (:609-637) turns the B per-utterance counts into the FM call(s), the
shared FlowMatchingModule (:1220-1377) integrates the student features and regresses the teacher's;
forward() returns router_weight * sum(router losses) + sum(flow losses) (:650-651) and the decoder
reads the LAST layer's FM output instead of the encoder output (:666).

On the engine all 16 layers run in one launch per kernel (csrc/encfm.hip): the router, the strategy
and the chain exchange the step counts through device memory, so the step has no host sync and
records into a step plan like the ver5 heads.  The f32 oracle is oracle/encfm.py (pinned by the
reference's own classes, tests/golden/kd_encfm.npz).
"""
from __future__ import annotations

import math

import torch

from . import _lib
from . import kernels as K
from .config import ENCFM_HIDDEN as HIDDEN
from .config import ENCFM_ROUTER_EMB as ROUTER_EMB
from .config import encfm_fixed_steps, encfm_specs

STRATEGIES = {"batch_mode": 0, "batch_avg": 1, "batch_median": 2, "group": 3}
SALT_ROUTER = 41      # counter-RNG stream of the router's Gumbel noise


def schedule_coeffs(cfg):
    """(ca, cv) per step count S = 1..max: nsx = ca x0 + cv v_last at t = 1/S (:1366-1367, :790-823)."""
    ca, cv = [], []
    for S in range(1, cfg.router_max_steps + 1):
        t = 1.0 / S
        if cfg.flow_schedule == "rectified":
            da, ds = 1.0, -1.0
        elif cfg.flow_schedule == "vp_ode":
            a, b = 19.9, 0.1
            al = math.exp(-0.25 * a * (1 - t) ** 2 - 0.5 * b * (1 - t))
            da = al * (0.5 * a * (1 - t) + 0.5 * b)
            ds = -al * da / math.sqrt(1 - al * al)
        else:
            raise ValueError(f"flow_schedule {cfg.flow_schedule!r}: ve_ode's dsigma/dt is 0 (asr_train.py:816-823), "
                             "its noise_scheduled_x divides by zero")
        ca.append(da / (-ds))
        cv.append(-1.0 / (-ds))
    import ctypes as C
    a, v = (C.c_float * len(ca))(*ca), (C.c_float * len(cv))(*cv)
    return a, v, C.cast(a, C.c_void_p), C.cast(v, C.c_void_p)


class EncFMWorkspace:
    """Per-(B, T) device buffers of the router, the strategy and the chain (saves sized for the maximum
    step count; the weight gradients read only the rows the strategy made active)."""

    def __init__(self, cfg, B, T, dev):
        L, Cs, Ct, Kmax, H = cfg.n_layers, cfg.d_student, cfg.d_teacher, cfg.router_max_steps, HIDDEN
        U = L * B
        n = U * T
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        self.B, self.T, self.n = B, T, n
        self.sv, self.tv, self.hcat, self.h0 = f(U, Cs), f(U, Ct), f(U, 2 * H + ROUTER_EMB), f(U, H)
        self.probs, self.ent = f(U, Kmax), f(U)
        self.steps = torch.empty(U, dtype=torch.int32, device=dev)
        self.S = torch.empty(U, dtype=torch.int32, device=dev)
        self.inv = f(U)
        self.off = torch.empty(U, dtype=torch.int64, device=dev)
        self.rows = torch.empty(1, dtype=torch.int64, device=dev)
        self.rloss, self.mean_steps, self.flow = f(L), f(L), f(L)
        self.stats = torch.zeros(4, device=dev)   # flow total, router_weight * router total, sum, mean steps
        self.c01 = f(2 * H)
        cap = Kmax * n
        bf = lambda *s: torch.empty(*s, dtype=torch.bfloat16, device=dev)  # noqa: E731
        self.X, self.A, self.DV, self.DA = bf(cap, 96), bf(cap, H), bf(cap, Cs), bf(cap, H)
        self.nsx, self.dtr = f(n, Cs), f(n, Ct)
        self.xS, self.gxS = f(B * T, Cs), f(B * T, Cs)
        self.dlogits, self.dh0, self.dhcat, self.dsv = f(U, Kmax), f(U, H), f(U, 2 * H + ROUTER_EMB), f(U, Cs)
        self._ca, self._cv, self.ca, self.cv = schedule_coeffs(cfg)   # host arrays + their pointers
        if not cfg.encfm_dynamic:
            self._fixed(cfg, dev)

    def _fixed(self, cfg, dev):
        """use_dynamic_steps=False: the per-layer step counts of sampling_steps_per_layer, else
        training_sampling (:639-645, config.encfm_fixed_steps), constant, so the strategy's outputs are
        computed once here."""
        L, B, T = cfg.n_layers, self.B, self.T
        steps = list(encfm_fixed_steps(cfg))
        S = [int(steps[u // B]) for u in range(L * B)]
        off, o = [], 0
        for s in S:
            off.append(o)
            o += s * T
        self.S.copy_(torch.tensor(S, dtype=torch.int32))
        self.off.copy_(torch.tensor(off, dtype=torch.int64))
        self.rows.fill_(o)
        self.inv.fill_(1.0 / (B * T * cfg.d_teacher))
        self.rloss.zero_()
        self.mean_steps.copy_(torch.tensor([float(s) for s in steps]))


def encfm_forward(cfg, P, sfeats, tfeats, ws: EncFMWorkspace, *, seed=None, train=True, gumbel=None,
                  bn_running=None):
    """All layers' router + strategy + FM chain.  sfeats (L, B*T, Cs), tfeats (L, B*T, Ct) stacked hook
    outputs.  Returns ws.xS (B*T, Cs): the last layer's FM output, the decoder's input.  ws.stats holds
    [sum flow losses, router_weight * sum router losses, their sum (forward's total_loss), mean steps];
    ws.flow / ws.rloss / ws.mean_steps the per-layer values (the reference's log keys)."""
    if cfg.encfm_meta != "mlp":
        from .fmmeta import meta_forward
        return meta_forward(cfg, P, sfeats, tfeats, ws, seed=seed, bn_running=bn_running, train=train)
    L, B, T = cfg.n_layers, ws.B, ws.T
    Cs, Ct, H, Kmax = cfg.d_student, cfg.d_teacher, HIDDEN, cfg.router_max_steps
    fm, r = "flow_matching.", "router."
    W1 = P[fm + "meta_encoder.0.weight"]
    K.call("kdfm_encfm_time_prep", K.ptr(W1), W1.stride(0), K.ptr(P[fm + "meta_encoder.0.bias"]),
           K.ptr(P[fm + "time_embed.weight"]), K.ptr(P[fm + "time_embed.bias"]), Cs, H, cfg.time_embed_dim,
           K.ptr(ws.c01), K._s())
    if cfg.encfm_dynamic:
        if gumbel is not None:
            assert gumbel.shape == (L * B, Kmax) and gumbel.is_contiguous()
        K.call("kdfm_encfm_router_fwd", K.ptr(sfeats), K.ptr(tfeats), K.ptr(P[r + "stu_proj.0.weight"]),
               K.ptr(P[r + "stu_proj.0.bias"]), K.ptr(P[r + "tch_proj.0.weight"]), K.ptr(P[r + "tch_proj.0.bias"]),
               K.ptr(P[r + "layer_emb.weight"]), K.ptr(P[r + "router.0.weight"]), K.ptr(P[r + "router.0.bias"]),
               K.ptr(P[r + "router.2.weight"]), K.ptr(P[r + "router.2.bias"]), K.ptr(gumbel), K.ptr(seed),
               SALT_ROUTER, 1 if train else 0, K.ptr(ws.sv), K.ptr(ws.tv), K.ptr(ws.hcat), K.ptr(ws.h0),
               K.ptr(ws.probs), K.ptr(ws.ent), K.ptr(ws.steps), L, B, T, Cs, Ct, Kmax, H, ROUTER_EMB, 1, K._s())
        K.call("kdfm_encfm_strategy", K.ptr(ws.steps), K.ptr(ws.ent), K.ptr(ws.S), K.ptr(ws.inv), K.ptr(ws.off),
               K.ptr(ws.rows), K.ptr(ws.rloss), K.ptr(ws.mean_steps), L, B, T, Kmax, Ct, STRATEGIES[cfg.encfm_strategy],
               8.0, 0.05, 0.001, 1 if train else 0, K._s())
    K.fill(ws.flow, 0.0)
    K.call("kdfm_encfm_chain_fwd", K.ptr(sfeats), K.ptr(tfeats), K.ptr(ws.S), K.ptr(ws.inv), K.ptr(ws.off),
           K.ptr(W1), W1.stride(0), K.ptr(ws.c01), K.ptr(P[fm + "meta_encoder.2.weight"]),
           K.ptr(P[fm + "meta_encoder.2.bias"]), K.ptr(P[fm + "shape_transformation_function.weight"]),
           K.ptr(P[fm + "shape_transformation_function.bias"]), ws.ca, ws.cv, Kmax,
           K.ptr(ws.X) if train else None, K.ptr(ws.A) if train else None, K.ptr(ws.nsx), K.ptr(ws.dtr),
           K.ptr(ws.xS), (L - 1) * B * T, K.ptr(ws.flow), L, B, T, Cs, Ct, K._s())
    if not train:   # the reference's flow loss is 0.0 outside training (asr_train.py:1363-1364)
        K.fill(ws.flow, 0.0)
    K.colsum(ws.flow.view(L, 1), ws.stats[0:1], accumulate=False)
    K.colsum(ws.rloss.view(L, 1), ws.stats[1:2], scale=cfg.router_weight, accumulate=False)
    K.colsum(ws.stats[0:2].view(2, 1), ws.stats[2:3], accumulate=False)
    K.colsum(ws.mean_steps.view(L, 1), ws.stats[3:4], scale=1.0 / L, accumulate=False)
    return ws.xS


def encfm_backward(cfg, P, G, ws: EncFMWorkspace, dfeats, gxS, wgrad_run, *, seed=None):
    """Data gradients into dfeats (L*B*T, Cs) (overwritten) from the flow losses, the router's entropy
    term and gxS (B*T, Cs) = d loss / d (last layer's FM output) through the decoder; the parameter
    gradients of flow_matching.* and router.* via `wgrad_run(fn, *keep)` (the weight-gradient stream)."""
    if cfg.encfm_meta != "mlp":
        from .fmmeta import meta_backward
        meta_backward(cfg, P, G, ws, dfeats, gxS, seed=seed)
        return
    L, B, T = cfg.n_layers, ws.B, ws.T
    Cs, Ct, H, Kmax = cfg.d_student, cfg.d_teacher, HIDDEN, cfg.router_max_steps
    fm, r = "flow_matching.", "router."
    W1 = P[fm + "meta_encoder.0.weight"]
    dsv = None
    if cfg.encfm_dynamic:
        coef = -cfg.router_weight * 0.001 / B   # d total / d H_u (entropy_weight 0.001, mean over the batch)
        K.call("kdfm_encfm_router_bwd", K.ptr(ws.probs), K.ptr(ws.hcat), K.ptr(ws.h0), K.ptr(P[r + "router.2.weight"]),
               K.ptr(P[r + "router.0.weight"]), K.ptr(P[r + "stu_proj.0.weight"]), float(coef), K.ptr(ws.dlogits),
               K.ptr(ws.dh0), K.ptr(ws.dhcat), K.ptr(ws.dsv), L, B, Cs, Kmax, K._s())
        dsv = ws.dsv
    K.call("kdfm_encfm_chain_bwd", K.ptr(ws.dtr), K.ptr(ws.A), K.ptr(gxS), (L - 1) * B * T, K.ptr(ws.S),
           K.ptr(ws.off), K.ptr(W1), W1.stride(0), K.ptr(P[fm + "meta_encoder.2.weight"]),
           K.ptr(P[fm + "shape_transformation_function.weight"]), ws.ca, ws.cv, Kmax, K.ptr(dsv), K.ptr(ws.DV),
           K.ptr(ws.DA), K.ptr(dfeats), L, B, T, Cs, Ct, K._s())
    cap = ws.X.shape[0]

    def weight_grads():
        gW1 = G[fm + "meta_encoder.0.weight"]
        # dW1x | dc0 | dc1 in columns 0 .. 95 of W1's gradient (the time-embedding columns are rewritten below)
        n = int(_lib.lib().kdfm_wgrad_bf16_ws(cap, H, 96, 0))
        wsb = K.scratch(ws.X.device, n)
        K.call("kdfm_wgrad_bf16_dev", K.ptr(ws.DA), K.ptr(ws.X), K.ptr(gW1), gW1.stride(0), None, cap, K.ptr(ws.rows),
               H, 96, 1.0, K.ptr(wsb), wsb.numel(), K._s())
        n = int(_lib.lib().kdfm_wgrad_bf16_ws(cap, Cs, H, 1))
        wsb = K.scratch(ws.X.device, n)
        gW2 = G[fm + "meta_encoder.2.weight"]
        K.call("kdfm_wgrad_bf16_dev", K.ptr(ws.DV), K.ptr(ws.A), K.ptr(gW2), gW2.stride(0),
               K.ptr(G[fm + "meta_encoder.2.bias"]), cap, K.ptr(ws.rows), Cs, H, 1.0, K.ptr(wsb), wsb.numel(), K._s())
        K.linear_dw(ws.dtr, ws.nsx, G[fm + "shape_transformation_function.weight"],
                    db=G[fm + "shape_transformation_function.bias"])
        if cfg.encfm_dynamic:   # L*B-row products: exact f32 (the router's forward is f32 too)
            K.linear_dw(ws.dlogits, ws.h0, G[r + "router.2.weight"], db=G[r + "router.2.bias"], math="f32")
            K.linear_dw(ws.dh0, ws.hcat, G[r + "router.0.weight"], db=G[r + "router.0.bias"], math="f32")
            K.linear_dw(ws.dhcat[:, :H], ws.sv, G[r + "stu_proj.0.weight"], db=G[r + "stu_proj.0.bias"], math="f32")
            K.linear_dw(ws.dhcat[:, H:2 * H], ws.tv, G[r + "tch_proj.0.weight"], db=G[r + "tch_proj.0.bias"],
                        math="f32")
        gemb = G[r + "layer_emb.weight"] if cfg.encfm_dynamic else ws.dsv   # ws.dsv: an unused sink when fixed
        K.wgrad_fold_flush()   # gW1 is read below: a deferred fold of the products above completes first
        K.call("kdfm_encfm_time_bwd", K.ptr(gW1), gW1.stride(0), K.ptr(G[fm + "meta_encoder.0.bias"]), K.ptr(W1),
               K.ptr(P[fm + "time_embed.weight"]), K.ptr(P[fm + "time_embed.bias"]), K.ptr(G[fm + "time_embed.weight"]),
               K.ptr(G[fm + "time_embed.bias"]), K.ptr(ws.dhcat), K.ptr(gemb), L if cfg.encfm_dynamic else 0, B, Cs,
               K._s())

    wgrad_run(weight_grads, ws.DA, ws.X, ws.DV, ws.A, ws.dtr, ws.nsx, ws.dlogits, ws.h0, ws.dh0, ws.hcat, ws.sv,
              ws.tv, ws.dhcat, ws.rows, W1)


__all__ = ["encfm_specs", "EncFMWorkspace", "encfm_forward", "encfm_backward", "STRATEGIES", "schedule_coeffs"]
