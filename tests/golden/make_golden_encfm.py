"""Golden vectors for the ENCODER-LEVEL flow matching with the DynamicStepRouter (asr_train.py's
DistilFlowMatchingCTCModelBPE, use_flow_matching=True, use_dynamic_steps=True) FROM THE REFERENCE'S
OWN CLASSES.

Runs only in the build container (needs /root/reference; never on the GPU box).  asr_train.py cannot
be imported (nemo / lightning / datasets at the top level), so the definitions are AST-selected from
/root/reference/asr_train.py -- DynamicStepRouter (:1021-1218), FlowMatchingModule (:1220-1377) and
the schedule functions (:790-823) -- and exec'd with {torch, nn, F}.  F.gumbel_softmax (the router's
training-mode sample, :1180) is replaced by the same formula on RECORDED Gumbel noise
(softmax((logits + g) / tau)), so the fixture is reproducible and the engine can be fed the same g.

The per-layer loop of DistilFlowMatchingCTCModelBPE.forward (:595-651) is restated below with the
module's attributes made explicit (it cannot be extracted: it lives inside forward() next to the NeMo
preprocessor / encoder calls): for every hooked layer i, router(s_i, t_i, layer_id=i) -> steps (B,),
router loss; the strategy picks the flow steps S (batch_mode: torch.mode, smallest on ties;
batch_avg: round(mean) clamped to [1, max]; batch_median: lower median; group: one FM call per
distinct S over that sub-batch); flow loss summed over layers; forward's total = router_weight *
sum(router losses) + sum(flow losses); the decoder then reads the LAST layer's FM output (:666).
Only numbers are written (kd_encfm.npz): inputs, noise, parameters, per-layer steps / S / losses, the
FM output, and gradients of the total plus a downstream term sum(fm_out * R) (standing in for the
decoder / CTC gradient that reaches fm_out) w.r.t. every parameter and every hooked student layer.

Usage:  python tests/golden/make_golden_encfm.py
"""
from __future__ import annotations

import ast
import os
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference/asr_train.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kd_encfm.npz")
KEEP_CLASSES = {"DynamicStepRouter", "FlowMatchingModule"}
KEEP_FUNCS = {"rectified_flow_schedule", "vp_ode_schedule", "ve_ode_schedule", "rectified_flow_schedule_deriv",
              "vp_ode_schedule_deriv", "ve_ode_schedule_deriv"}
STRATEGIES = ("batch_mode", "batch_avg", "batch_median", "group")


class _FWithRecordedGumbel(types.ModuleType):
    """Proxy for `F` inside the exec'd reference code: gumbel_softmax uses recorded noise."""

    def __init__(self):
        super().__init__("F_proxy")
        self.queue = []

    def __getattr__(self, name):
        return getattr(F, name)

    def gumbel_softmax(self, logits, tau=1.0, hard=False, dim=-1):
        assert not hard
        g = self.queue.pop(0)
        assert g.shape == logits.shape
        return F.softmax((logits + g) / tau, dim=dim)


def load_reference():
    tree = ast.parse(open(REF).read())
    body = [n for n in tree.body if (isinstance(n, ast.ClassDef) and n.name in KEEP_CLASSES)
            or (isinstance(n, ast.FunctionDef) and n.name in KEEP_FUNCS)]
    proxy = _FWithRecordedGumbel()
    ns = {"torch": torch, "nn": nn, "F": proxy}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF, "exec"), ns)
    return ns, proxy


def run(ns, proxy, strategy, L, B, T, seed):
    Cs, Ct, maxS = 88, 176, 8
    torch.manual_seed(seed)
    flow_cfg = {"meta_encoder_type": "mlp", "feature_dim": Cs, "time_embed_dim": 32, "hidden_dim": 128,
                "training_sampling": 8, "inference_sampling": 8, "weight": 1.0, "noise_schedule": "rectified",
                "loss": "mse", "shape_transform": "linear", "student_dim": Cs, "teacher_dim": Ct,
                "student_head_num": 2, "teacher_head_num": 4}
    fm = ns["FlowMatchingModule"](flow_cfg).train()
    # DistilFlowMatchingCTCModelBPE.__init__ (:511-518), router_max_sampling_steps = 8 (args default)
    router = ns["DynamicStepRouter"](max_steps=maxS, min_steps=1, stu_dim=Cs, tch_dim=Ct, use_layer_id=True,
                                     num_layers=L, layer_emb_dim=32, temperature=1.0, budget_target=8.0,
                                     budget_weight=0.05, entropy_weight=0.001).train()
    router_weight = 1.0
    s = [(0.5 * torch.randn(B, T, Cs)).requires_grad_(True) for _ in range(L)]   # hook layout (B, T, C)
    t = [torch.randn(B, T, Ct) for _ in range(L)]
    gum = [-torch.empty(B, maxS).exponential_().log() for _ in range(L)]
    R = torch.randn(B, T, Cs)
    proxy.queue.extend(gum)
    total_flow = torch.zeros(())
    total_router = torch.zeros(())
    steps_all, S_all, flow_all, rl_all = [], [], [], []
    fm_out = None
    for i in range(L):
        steps_b, rloss, aux = router(s[i], t[i], layer_id=i)
        total_router = total_router + rloss
        if strategy == "batch_mode":
            S = int(torch.mode(steps_b).values.item())
        elif strategy == "batch_avg":
            S = int(torch.round(steps_b.float().mean()).clamp(1, maxS).item())
        elif strategy == "batch_median":
            S = int(torch.median(steps_b.float()).clamp(1, maxS).item())
        else:
            S = 0
        if strategy != "group":
            fl, fm_out = fm(s[i], t[i], layer_sampling_step=S, layer_id=i)
            total_flow = total_flow + fl
            flow_all.append(float(fl.detach()))
        else:
            fm_out = torch.zeros_like(s[i])
            fl_sum = torch.zeros(())
            for sv in torch.unique(steps_b).tolist():
                idx = steps_b == sv
                fl_s, out_s = fm(s[i][idx], t[i][idx], layer_sampling_step=int(sv), layer_id=i)
                fm_out[idx] = out_s
                fl_sum = fl_sum + fl_s
            total_flow = total_flow + fl_sum
            flow_all.append(float(fl_sum.detach()))
        steps_all.append(steps_b.numpy().astype(np.int64))
        S_all.append(S)
        rl_all.append(float(rloss.detach()))
    total = total_router * router_weight + total_flow
    objective = total + (fm_out * R).sum()
    params = {"flow_matching." + n: p for n, p in fm.named_parameters()}
    params.update({"router." + n: p for n, p in router.named_parameters()})
    names = list(params)
    grads = torch.autograd.grad(objective, [params[n] for n in names] + s, allow_unused=True)
    pre = strategy + "."
    shared = {}
    for i in range(L):
        shared[f"in.s{i}"] = s[i].detach().numpy()
        shared[f"in.t{i}"] = t[i].numpy()
        shared[f"in.gumbel{i}"] = gum[i].numpy()
    shared["in.R"] = R.numpy()
    for n in names:
        shared["param." + n] = params[n].detach().numpy()
    arrays = {pre + "total": np.array(float(total.detach()), dtype=np.float64),
              pre + "flow": np.array(flow_all, dtype=np.float64), pre + "router_loss": np.array(rl_all, dtype=np.float64),
              pre + "steps": np.stack(steps_all), pre + "S": np.array(S_all, dtype=np.int64),
              pre + "fm_out": fm_out.detach().numpy()}
    for i in range(L):
        arrays[pre + f"grad.s{i}"] = grads[len(names) + i].numpy()
    for n, g in zip(names, grads[:len(names)]):
        arrays[pre + "grad." + n] = np.zeros(params[n].shape, np.float32) if g is None else g.numpy()
    return arrays, shared


def main(L=2, B=4, T=17, seed=31):
    """Every strategy on the same inputs, noise and parameters (same seed): shared arrays stored once."""
    ns, proxy = load_reference()
    arrays = {"meta.L": np.array(L), "meta.B": np.array(B), "meta.T": np.array(T)}
    for strategy in STRATEGIES:
        got, shared = run(ns, proxy, strategy, L, B, T, seed=seed)
        arrays.update(got)
        arrays.update(shared)
        print(strategy, "S per layer", arrays[strategy + ".S"].tolist(), "total", float(arrays[strategy + ".total"]))
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
