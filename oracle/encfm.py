"""CPU oracle (TEST INFRASTRUCTURE ONLY -- never imported by the product path) for the ENCODER-LEVEL
flow matching of asr_train.py's DistilFlowMatchingCTCModelBPE (use_flow_matching=True,
use_dynamic_steps=True): the DynamicStepRouter, the step-count strategies and the FlowMatchingModule
applied to every hooked Conformer layer, plus the decoder reading the last layer's FM output.

A plain-PyTorch restatement (autograd supplies the gradients), pinned by tests/golden/kd_encfm.npz,
which make_golden_encfm.py produced from the reference's own DynamicStepRouter / FlowMatchingModule
classes (tests/test_oracle_encfm.py).  Citations are /root/reference/asr_train.py line numbers.

Parameter names follow the reference module tree: flow_matching.{time_embed, meta_encoder.0,
meta_encoder.2, shape_transformation_function}.*, router.{stu_proj.0, tch_proj.0, layer_emb, router.0,
router.2}.*.  Features are in the hook layout (B, T, C).
"""
from __future__ import annotations

import math

import torch

STRATEGIES = ("batch_mode", "batch_avg", "batch_median", "group")


def _lin(x, P, name):
    return x @ P[name + ".weight"].t() + P[name + ".bias"]


def router_forward(P, s, t, layer_id, gumbel, tau=1.0, budget_target=8.0, budget_weight=0.05,
                   entropy_weight=0.001, min_steps=1):
    """DynamicStepRouter.forward in training mode (:1131-1218).  The time axis is reduced by a plain
    mean over all T frames (feature_reduce 'gap', :1121-1129; padding included, as the hooks hand the
    padded features over).  steps = argmax(softmax((logits + g) / tau)) + 1 = argmax(logits + g) + 1
    (the straight-through y is unused by the caller, :603); loss = budget_weight (mean(steps) -
    budget_target)^2 (no gradient: steps are integers) - entropy_weight * mean_b H(softmax(logits))."""
    B = s.shape[0]
    sv = s.mean(dim=1)
    tv = t.mean(dim=1)
    sh = torch.relu(_lin(sv, P, "router.stu_proj.0"))
    th = torch.relu(_lin(tv, P, "router.tch_proj.0"))
    emb = P["router.layer_emb.weight"][layer_id].expand(B, -1)
    h = torch.cat([sh, th, emb], dim=-1)
    logits = _lin(torch.relu(_lin(h, P, "router.router.0")), P, "router.router.2")
    K = logits.shape[-1]
    if min_steps > 1:
        mask = torch.zeros(K, dtype=logits.dtype)
        mask[:min_steps - 1] = float("-inf")
        logits = logits + mask
    probs = torch.softmax(logits, dim=-1)
    steps = torch.argmax(logits + gumbel, dim=-1) + 1
    loss = logits.new_zeros(())
    if budget_target is not None and budget_weight > 0:
        loss = loss + budget_weight * (steps.to(logits.dtype).mean() - budget_target) ** 2
    if entropy_weight > 0:
        ent = -(probs * probs.clamp_min(1e-8).log()).sum(-1).mean()
        loss = loss - entropy_weight * ent
    return steps, loss, probs


def choose_steps(steps, strategy, max_steps):
    """The layer's flow step count from the per-utterance router steps (:609-625): batch_mode = the most
    frequent value (smallest on ties, torch.mode on the CPU); batch_avg = round-half-even of the mean,
    clamped; batch_median = the lower median, clamped."""
    if strategy == "batch_mode":
        vals, counts = torch.unique(steps, return_counts=True)
        return int(vals[torch.argmax(counts)])   # unique is sorted: the first maximum is the smallest value
    if strategy == "batch_avg":
        return int(min(max(round(float(steps.double().mean())), 1), max_steps))
    if strategy == "batch_median":
        srt = torch.sort(steps).values
        return int(min(max(int(srt[(len(srt) - 1) // 2]), 1), max_steps))
    raise ValueError(strategy)


def schedule_coeffs(S, schedule="rectified", vp=(19.9, 0.1)):
    """noise_scheduled_x = (dalpha * s_f - v) / (-dsigma) at the last loop time t = 1/S (:1366-1367;
    schedules :790-823).  Returns (ca, cv) with nsx = ca * s_f + cv * v."""
    tt = 1.0 / S
    if schedule == "rectified":
        da, ds = 1.0, -1.0
    elif schedule == "vp_ode":
        a, b = vp
        al = math.exp(-0.25 * a * (1 - tt) ** 2 - 0.5 * b * (1 - tt))
        da = al * (0.5 * a * (1 - tt) + 0.5 * b)
        ds = -al * da / math.sqrt(1 - al * al)
    else:
        raise ValueError(f"schedule {schedule!r}: ve_ode has dsigma/dt = 0 (:816-823), a division by zero")
    return da / (-ds), -1.0 / (-ds)


def _layer_norm(x, P, name, eps=1e-5):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], eps)


def _mha(x, P, name, heads):
    """nn.MultiheadAttention(x, x, x) core, batch-first (B, T, C), no masks, dropout off (:847, :968)."""
    B, T, C = x.shape
    dk = C // heads
    qkv = x @ P[name + ".in_proj_weight"].t() + P[name + ".in_proj_bias"]
    q, k, v = (qkv[..., j * C:(j + 1) * C].reshape(B, T, heads, dk).transpose(1, 2) for j in range(3))
    att = torch.softmax((q / math.sqrt(dk)) @ k.transpose(-1, -2), dim=-1)
    return _lin((att @ v).transpose(1, 2).reshape(B, T, C), P, name + ".out_proj")


def _conformer_meta(P, e, heads, bn_state=None, momentum=0.1, eps=1e-5):
    """ConformerEncoder (:1000-1020) with dropouts off: input_proj, then 4 ConformerBlocks (:962-999),
    each FF1 half step (norm_ff1 then the module's own LN, Linear -> SiLU -> Linear), MHA on mha_layer(x),
    ConvModule (:932-961: LN -> pointwise_conv1 -> depthwise k=31 pad 15 -> BatchNorm1d with batch
    statistics -> SiLU -> pointwise_conv2), FF2 half step, norm_final.  bn_state: {buffer name: tensor}
    running statistics updated in place per call (training mode, unbiased variance, momentum 0.1)."""
    me = "flow_matching.meta_encoder."
    F_ = torch.nn.functional
    x = _lin(e, P, me + "input_proj")
    for l in range(4):
        p = f"{me}layers.{l}."

        def ff(y, name):
            y = _layer_norm(y, P, p + name + ".net.0")
            return _lin(F_.silu(_lin(y, P, p + name + ".net.1")), P, p + name + ".net.4")

        x = x + 0.5 * ff(_layer_norm(x, P, p + "norm_ff1"), "ff1")
        x = x + _mha(_layer_norm(x, P, p + "mha_layer"), P, p + "mha", heads)
        c = p + "conv_module."
        y = _layer_norm(x, P, c + "layer_norm").transpose(1, 2)
        y = F_.conv1d(y, P[c + "pointwise_conv1.weight"], P[c + "pointwise_conv1.bias"])
        C2 = y.shape[1]
        y = F_.conv1d(y, P[c + "depthwise_conv.weight"], P[c + "depthwise_conv.bias"], padding=15, groups=C2)
        mean = y.mean(dim=(0, 2))
        var = y.var(dim=(0, 2), unbiased=False)
        if bn_state is not None:
            n = y.shape[0] * y.shape[2]
            rm, rv = bn_state[c + "batch_norm.running_mean"], bn_state[c + "batch_norm.running_var"]
            rm.mul_(1 - momentum).add_(momentum * mean.detach())
            rv.mul_(1 - momentum).add_(momentum * var.detach() * n / (n - 1))
        y = (y - mean[None, :, None]) / torch.sqrt(var[None, :, None] + eps)
        y = y * P[c + "batch_norm.weight"][None, :, None] + P[c + "batch_norm.bias"][None, :, None]
        y = F_.conv1d(F_.silu(y), P[c + "pointwise_conv2.weight"], P[c + "pointwise_conv2.bias"])
        x = x + y.transpose(1, 2)
        x = x + 0.5 * ff(_layer_norm(x, P, p + "norm_ff2"), "ff2")
        x = _layer_norm(x, P, p + "norm_final")
    return x


def meta_velocity(P, e, meta="mlp", heads=2, bn_state=None):
    """FlowMatchingModule.meta_encoder on e = [x; te(t)] (B, T, Cs+E) -> v (B, T, Cs) (:1244-1259, 1328-1345).
    mlp: W2 relu(W1 e + b1) + b2.  cnn: Conv1d(k=3, pad 1 per utterance) -> ReLU -> Conv1d(k=1) over the
    frames.  swin (SwinTransformerEncoder :844-866): nn.MultiheadAttention(e, e, e) over the T frames of
    each utterance (no mask, `heads` heads, q scaled by 1/sqrt(dk)), out_proj, then linear2 relu(linear1)."""
    me = "flow_matching.meta_encoder."
    if meta == "mlp":
        return _lin(torch.relu(_lin(e, P, me + "0")), P, me + "2")
    if meta == "cnn":
        a = torch.relu(torch.nn.functional.conv1d(e.transpose(1, 2), P[me + "0.weight"], P[me + "0.bias"], padding=1))
        return torch.nn.functional.conv1d(a, P[me + "2.weight"], P[me + "2.bias"]).transpose(1, 2)
    if meta == "swin":
        B, T, C = e.shape
        dk = C // heads
        qkv = e @ P[me + "attn.in_proj_weight"].t() + P[me + "attn.in_proj_bias"]
        q, k, v = (qkv[..., j * C:(j + 1) * C].reshape(B, T, heads, dk).transpose(1, 2) for j in range(3))
        att = torch.softmax((q / math.sqrt(dk)) @ k.transpose(-1, -2), dim=-1)
        o = (att @ v).transpose(1, 2).reshape(B, T, C)
        ao = _lin(o, P, me + "attn.out_proj")
        return _lin(torch.relu(_lin(ao, P, me + "linear1")), P, me + "linear2")
    if meta == "conformer":
        return _conformer_meta(P, e, heads, bn_state)
    if meta == "unet":
        return _unet_meta(P, e)
    raise ValueError(f"meta-encoder {meta!r} not in the oracle (mlp, cnn, swin, conformer, unet)")


def _unet_meta(P, e, num_layers=4):
    """UNet1D (asr_train.py:880-917) over the frames of each utterance, e (B, T, Cin) -> (B, T', Cs): num_layers
    Conv1d(k 4, stride 2, pad 1) downs (each output kept as a skip), Conv1d(k 3, pad 1) bottleneck, then per
    skip (deepest first) zero-pad x at the end to the skip's length, concatenate [x | skip] on channels and
    ConvTranspose1d(k 4, stride 2, pad 1); Conv1d(k 1) final.  T' = 2 floor(T / 2): odd T gives T - 1 frames
    (the reference's update x - v / S then fails to broadcast -- fm_forward raises likewise)."""
    me = "flow_matching.meta_encoder."
    F = torch.nn.functional
    x = e.transpose(1, 2)
    skips = []
    for i in range(num_layers):
        x = F.conv1d(x, P[me + f"downs.{i}.weight"], P[me + f"downs.{i}.bias"], stride=2, padding=1)
        skips.append(x)
    x = F.conv1d(x, P[me + "bottleneck.weight"], P[me + "bottleneck.bias"], padding=1)
    for i in range(num_layers):
        skip = skips.pop()
        if x.shape[2] != skip.shape[2]:
            x = F.pad(x, (0, skip.shape[2] - x.shape[2]))
        x = F.conv_transpose1d(torch.cat([x, skip], dim=1), P[me + f"ups.{i}.weight"], P[me + f"ups.{i}.bias"],
                               stride=2, padding=1)
    return F.conv1d(x, P[me + "final.weight"], P[me + "final.bias"]).transpose(1, 2)


def fm_forward(P, x0, tf, S, schedule="rectified", meta="mlp", heads=2, bn_state=None):
    """FlowMatchingModule.forward, shape_transform 'linear', loss 'mse' (:1318-1377): for i = S..1,
    t = i/S: v = meta_encoder([x; te(t)]) (meta_velocity), x <- x - v/S; then
    loss = mean((Wst nsx + bst - t_f)^2) with nsx from the LAST velocity and the ORIGINAL input.
    x0: (B, T, Cs), tf: (B, T, Ct).  Returns (loss, x_S)."""
    x = x0
    v = None
    for i in range(S, 0, -1):
        tt = torch.full(x0.shape[:-1] + (1,), i / S, dtype=x0.dtype)
        te = _lin(tt, P, "flow_matching.time_embed")
        v = meta_velocity(P, torch.cat([x, te], dim=-1), meta, heads, bn_state)
        x = x - v / S
    ca, cv = schedule_coeffs(S, schedule)
    nsx = ca * x0 + cv * v
    tr = _lin(nsx, P, "flow_matching.shape_transformation_function")
    return ((tr - tf) ** 2).mean(), x


def encfm_fixed_forward(P, sfeats, tfeats, steps, schedule="rectified", meta="mlp", heads=2, bn_state=None):
    """use_dynamic_steps=False with sampling_steps_per_layer (:639-641): no router, layer i runs steps[i]
    FM steps; same result dict as encfm_forward (router losses 0)."""
    flows = []
    fm_out = None
    for i, (s, t) in enumerate(zip(sfeats, tfeats)):
        fl, fm_out = fm_forward(P, s, t, int(steps[i]), schedule, meta, heads, bn_state)
        flows.append(fl)
    total = sum(flows[1:], flows[0])
    B = sfeats[0].shape[0]
    return {"total": total, "flow": flows, "router_loss": [total.new_zeros(()) for _ in flows],
            "steps": torch.tensor([[int(S)] * B for S in steps]), "S": [int(S) for S in steps], "fm_out": fm_out}


def encfm_forward(P, sfeats, tfeats, gumbels, strategy="batch_mode", max_steps=8, router_weight=1.0,
                  tau=1.0, schedule="rectified"):
    """The flow-matching block of DistilFlowMatchingCTCModelBPE.forward (:595-666) over the hooked layer
    pairs (lists of (B, T, C)): returns dict(total = router_weight * sum router losses + sum flow losses,
    flow (per layer), router_loss (per layer), steps (L, B), S (per layer; 0 for 'group'), fm_out = the
    last layer's FM output, which replaces the encoder output as the decoder input, :666)."""
    total_flow = sfeats[0].new_zeros(())
    total_router = sfeats[0].new_zeros(())
    flows, rls, steps_all, S_all = [], [], [], []
    fm_out = None
    for i, (s, t) in enumerate(zip(sfeats, tfeats)):
        steps, rl, _ = router_forward(P, s, t, i, gumbels[i], tau=tau)
        total_router = total_router + rl
        if strategy == "group":
            fm_out = torch.zeros_like(s)
            fl = s.new_zeros(())
            for sv in torch.unique(steps).tolist():
                idx = steps == sv
                f, o = fm_forward(P, s[idx], t[idx], int(sv), schedule)
                fm_out = fm_out.index_put((idx.nonzero()[:, 0],), o)
                fl = fl + f
            S = 0
        else:
            S = choose_steps(steps, strategy, max_steps)
            fl, fm_out = fm_forward(P, s, t, S, schedule)
        total_flow = total_flow + fl
        flows.append(fl)
        rls.append(rl)
        steps_all.append(steps)
        S_all.append(S)
    return {"total": router_weight * total_router + total_flow, "flow": flows, "router_loss": rls,
            "steps": torch.stack(steps_all), "S": S_all, "fm_out": fm_out}


def init_encfm(Cs=88, Ct=176, L=16, hidden=128, time_dim=32, proj=128, rhidden=128, K=8, layer_emb=32, seed=0):
    """nn.Linear / nn.Embedding default initialisation shapes for the two modules (:1240-1292, :1076-1098)."""
    g = torch.Generator().manual_seed(seed)

    def lin(name, o, i):
        bound = 1.0 / math.sqrt(i)
        return {name + ".weight": (torch.rand(o, i, generator=g) * 2 - 1) * bound,
                name + ".bias": (torch.rand(o, generator=g) * 2 - 1) * bound}
    P = {}
    P.update(lin("flow_matching.time_embed", time_dim, 1))
    P.update(lin("flow_matching.meta_encoder.0", hidden, Cs + time_dim))
    P.update(lin("flow_matching.meta_encoder.2", Cs, hidden))
    P.update(lin("flow_matching.shape_transformation_function", Ct, Cs))
    P.update(lin("router.stu_proj.0", proj, Cs))
    P.update(lin("router.tch_proj.0", proj, Ct))
    P["router.layer_emb.weight"] = torch.randn(L, layer_emb, generator=g)
    P.update(lin("router.router.0", rhidden, 2 * proj + layer_emb))
    P.update(lin("router.router.2", K, rhidden))
    return P


__all__ = ["router_forward", "choose_steps", "schedule_coeffs", "fm_forward", "encfm_forward", "init_encfm",
           "STRATEGIES"]
