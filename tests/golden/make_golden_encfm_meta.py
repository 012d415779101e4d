"""Golden vectors for the encoder-level FlowMatchingModule's OTHER meta-encoders (asr_train.py:1241-1277:
"cnn", "swin", "conformer", "unet"; the flowkd_<meta>_linear_* launchers) FROM THE REFERENCE'S OWN CLASSES.

Runs only in the build container (needs /root/reference; never on the GPU box).  As in
make_golden_encfm.py the classes are AST-selected from /root/reference/asr_train.py -- FlowMatchingModule
(:1220-1377), SwinTransformerEncoder (:844-866), UNet1D (:880-917), FeedForwardModule / ConvModule /
ConformerBlock / ConformerEncoder (:918-1020) and the schedule functions -- and exec'd with {torch, nn, F}.
The fixed-step path is used (use_dynamic_steps False with sampling_steps_per_layer; the router is
exercised by kd_encfm.npz): per hooked layer i, FM(s_i, t_i, S_i) -> (flow loss, x_S), losses summed, and
a downstream term sum(x_S(last layer) * R) stands in for the decoder's gradient.  The conformer
meta-encoder's dropouts (0.1, :918-1013) are switched off for the fixture (the engine's parity mode runs
dropout 0 too); its BatchNorm uses batch statistics (training mode).  Written: inputs, parameters, losses,
the FM output and the gradients of the objective w.r.t. every parameter and every hooked student layer.
Combinations the reference cannot run are NOT fixtures (tests/golden/README-style notes in DESIGN.md):
shape_transform "conv1d" applies Conv1d(88, 176, 1) to a (B, T, 88) tensor (RuntimeError unless T == 88),
loss "cosine" calls CosineEmbeddingLoss without its target (TypeError), "unet" with an odd frame count
returns T-1 frames and the update x - v / S fails to broadcast.  "unet" (UNet1D, :880-917) is written at an
EVEN frame count (T = 36: its skip lengths 18, 9, 4, 2 exercise the up path's zero pad) with hidden_dim 8 (the
U-Net's base width: 8 .. 64 channels instead of 128 .. 1024 keeps the fixture small; the layer structure is
the same), under "unet.*" with its own "unet.meta.T" / "unet.meta.hidden".

Usage:  python tests/golden/make_golden_encfm_meta.py
"""
from __future__ import annotations

import ast
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference/asr_train.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kd_encfm_meta.npz")
KEEP_CLASSES = {"FlowMatchingModule", "SwinTransformerEncoder", "UNet1D", "FeedForwardModule", "ConvModule",
                "ConformerBlock", "ConformerEncoder", "MLPEncoder", "CNNEncoder"}
KEEP_FUNCS = {"rectified_flow_schedule", "vp_ode_schedule", "ve_ode_schedule", "rectified_flow_schedule_deriv",
              "vp_ode_schedule_deriv", "ve_ode_schedule_deriv"}
METAS = ("cnn", "swin", "conformer")


def seeded_params(module, seed):
    """Overwrite every parameter (named_parameters order) with values the GPU test regenerates without the
    reference: >= 2-D U(-1/sqrt(fan_in), 1/sqrt(fan_in)); 1-D scales (names ending in 'weight': LayerNorm /
    BatchNorm) 1 + 0.1 U(-1, 1); other 1-D (biases) 0.1 U(-1, 1); one CPU generator per tensor."""
    with torch.no_grad():
        for i, (name, p) in enumerate(module.named_parameters()):
            g = torch.Generator().manual_seed(seed * 1000 + i)
            u = torch.rand(p.shape, generator=g) * 2 - 1
            if p.dim() >= 2:
                p.copy_(u / (p[0].numel() ** 0.5))
            elif name.endswith("weight"):
                p.copy_(1.0 + 0.1 * u)
            else:
                p.copy_(0.1 * u)


def load_reference():
    tree = ast.parse(open(REF).read())
    body = [n for n in tree.body if (isinstance(n, ast.ClassDef) and n.name in KEEP_CLASSES)
            or (isinstance(n, ast.FunctionDef) and n.name in KEEP_FUNCS)]
    ns = {"torch": torch, "nn": nn, "F": F}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF, "exec"), ns)
    return ns


def run(ns, meta, L, B, T, steps, seed, hidden=128):
    Cs, Ct = 88, 176
    torch.manual_seed(seed)
    flow_cfg = {"meta_encoder_type": meta, "time_embed_dim": 32, "hidden_dim": hidden, "training_sampling": 8,
                "inference_sampling": 8, "weight": 1.0, "noise_schedule": "rectified", "loss": "mse",
                "shape_transform": "linear", "student_dim": Cs, "teacher_dim": Ct, "student_head_num": 2,
                "teacher_head_num": 4}
    torch.manual_seed(seed)
    fm = ns["FlowMatchingModule"](flow_cfg).train()
    seeded_params(fm, seed)
    for m in fm.modules():   # parity fixture: dropout off (conformer meta-encoder only has dropouts)
        if isinstance(m, nn.Dropout):
            m.p = 0.0
        if isinstance(m, nn.MultiheadAttention):
            m.dropout = 0.0
    gi = torch.Generator().manual_seed(seed + 99)
    s = [(0.5 * torch.randn(B, T, Cs, generator=gi)).requires_grad_(True) for _ in range(L)]
    t = [torch.randn(B, T, Ct, generator=gi) for _ in range(L)]
    R = torch.randn(B, T, Cs, generator=gi)
    total = torch.zeros(())
    flows = []
    out = None
    for i in range(L):
        fl, out = fm(s[i], t[i], layer_sampling_step=int(steps[i]), layer_id=i)
        total = total + fl
        flows.append(float(fl.detach()))
    objective = total + (out * R).sum()
    params = {"flow_matching." + n: p for n, p in fm.named_parameters()}
    names = list(params)
    grads = torch.autograd.grad(objective, [params[n] for n in names] + s, allow_unused=True)
    pre = meta + "."
    arrays = {pre + "total": np.array(float(total.detach()), dtype=np.float64),
              pre + "flow": np.array(flows, dtype=np.float64), pre + "fm_out": out.detach().numpy(),
              pre + "names": np.array(names), pre + "shapes": np.array([str(tuple(params[n].shape)) for n in names])}
    for i in range(L):   # inputs: regenerated from (seed + 99) in the test; gradients stored
        arrays[pre + f"grad.s{i}"] = grads[len(names) + i].numpy()
    for n, g in zip(names, grads[:len(names)]):   # parameters: regenerated by seeded_params in the test
        arrays[pre + "grad." + n] = np.zeros(params[n].shape, np.float32) if g is None else g.numpy()
    for n, b in fm.named_buffers():   # BatchNorm running stats after the step (conformer)
        arrays[pre + "buffer.flow_matching." + n] = b.detach().numpy()
    return arrays


def main(L=2, B=2, T=32, steps=(2, 3), seed=7):
    ns = load_reference()
    arrays = {"meta.L": np.array(L), "meta.B": np.array(B), "meta.T": np.array(T), "meta.steps": np.array(steps)}
    for meta in METAS:
        got = run(ns, meta, L, B, T, steps, seed)
        arrays.update(got)
        print(meta, "params", len(got[meta + ".names"]), "total", float(got[meta + ".total"]))
    unet_T, unet_hidden = 36, 8
    got = run(ns, "unet", L, B, unet_T, steps, seed, hidden=unet_hidden)
    arrays.update(got)
    arrays.update({"unet.meta.T": np.array(unet_T), "unet.meta.hidden": np.array(unet_hidden)})
    print("unet params", len(got["unet.names"]), "total", float(got["unet.total"]))
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
