"""Generate golden vectors for the ver5 KD heads FROM THE REFERENCE'S OWN CLASSES.

Runs only in the survey/build container (needs /root/reference; never on the GPU box).
`import asr_train_diffm` fails there on its top-level nemo/lightning/ruamel imports, so this
script parses /root/reference/asr_train_diffm.py with `ast`, keeps only the class/function
definitions the ver5 heads need (asr_train_diffm.py:400-497 heads, :840-873 schedules,
:1270-1427 FlowMatchingModule, and the method _compute_v_losses_one_layer :645-729) and execs
them with {torch, nn, F}.  NoiseAdapter's torch.randn_like draw is replaced by a recorded noise
tensor so the fixture is reproducible.  Nothing from the reference is written to the repo except
the resulting numbers (inputs, parameters, outputs, gradients) in kd_heads_ver5.npz.

Usage:  python tests/golden/make_golden.py
  -> kd_heads_ver5.npz (B=2, T'=29) and kd_heads_ver5_b1t401.npz (one benchmark-shape layer: B=1,
     T'=401 = 16.0 s of audio after 4x subsampling)
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference/asr_train_diffm.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kd_heads_ver5.npz")

KEEP_CLASSES = {"TeacherAutoEncoder", "StudentProjector", "NoiseAdapter", "SimpleDenoiser", "FMLatent",
                "FlowMatchingModule"}
KEEP_FUNCS = {"rectified_flow_schedule", "rectified_flow_schedule_deriv"}


class _TorchWithInjectedNoise(types.ModuleType):
    """Proxy for `torch` inside the exec'd reference code: randn_like pops recorded noise."""

    def __init__(self):
        super().__init__("torch_proxy")
        self.queue = []

    def __getattr__(self, name):
        return getattr(torch, name)

    def randn_like(self, x, *a, **k):
        e = self.queue.pop(0)
        assert e.shape == x.shape, (e.shape, x.shape)
        return e.clone()


def load_reference():
    src = open(REF).read()
    tree = ast.parse(src)
    body = []
    method = None
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name in KEEP_CLASSES:
            body.append(node)
        elif isinstance(node, ast.FunctionDef) and node.name in KEEP_FUNCS:
            body.append(node)
        elif isinstance(node, ast.ClassDef) and node.name == "DistilFlowMatchingCTCModelBPE":
            for sub in node.body:
                if isinstance(sub, ast.FunctionDef) and sub.name in ("_compute_v_losses_one_layer", "_BHT_to_BTH"):
                    body.append(sub)
    mod = ast.Module(body=body, type_ignores=[])
    proxy = _TorchWithInjectedNoise()
    ns = {"torch": proxy, "nn": nn, "F": F}
    exec(compile(mod, REF, "exec"), ns)
    return ns, proxy


def main(B=2, T=29, seed=7, out_path=OUT, extras=True):
    ns, proxy = load_reference()
    torch.manual_seed(seed)
    Cs, Ct, L = 88, 176, 96
    flow_cfg = {"meta_encoder_type": "mlp", "feature_dim": Cs, "time_embed_dim": 32, "hidden_dim": L,
                "training_sampling": 8, "inference_sampling": 8, "weight": 1.0, "noise_schedule": "rectified",
                "loss": "mse", "shape_transform": "linear", "student_dim": Cs, "teacher_dim": Ct,
                "student_head_num": 2, "teacher_head_num": 4}

    class Heads(nn.Module):   # the attributes DistilFlowMatchingCTCModelBPE.__init__ builds (:553-564)
        def __init__(self):
            super().__init__()
            self.version = 5
            self.recon_crit = nn.MSELoss()
            self.kd_crit = nn.MSELoss()
            self.tae = ns["TeacherAutoEncoder"](teacher_dim=Ct, latent_dim=L)
            self.sproj = ns["StudentProjector"](student_dim=Cs, latent_dim=L)
            self.adapter = ns["NoiseAdapter"](latent_dim=L)
            self.denoiser = ns["SimpleDenoiser"](latent_dim=L, steps=9)
            self.fm_latent = ns["FMLatent"](latent_dim=L, flow_cfg=flow_cfg)
            self.fm_latent_2 = ns["FMLatent"](latent_dim=L, flow_cfg=flow_cfg)

    Heads._BHT_to_BTH = staticmethod(ns["_BHT_to_BTH"])
    Heads._compute_v_losses_one_layer = ns["_compute_v_losses_one_layer"]
    heads = Heads().train()
    s = torch.randn(B, T, Cs, requires_grad=True)    # hook output layout (B,T,C)
    t = torch.randn(B, T, Ct)
    eps = torch.randn(B, L, T)
    proxy.queue.append(eps)
    out = heads._compute_v_losses_one_layer(s, t)
    total = out["recon_loss"] + out["fm_loss_post"]
    params = dict(heads.named_parameters())
    names = [n for n in params if not n.startswith("fm_latent_2.")]
    grads = torch.autograd.grad(total, [params[n] for n in names] + [s])
    arrays = {"in.s": s.detach().numpy(), "in.t": t.numpy(), "in.eps": eps.numpy(),
              "out.recon": np.array(out["recon_loss"].item(), dtype=np.float64),
              "out.fm_post": np.array(out["fm_loss_post"].item(), dtype=np.float64),
              "grad.in.s": grads[-1].numpy()}
    for n, p in params.items():
        arrays["param." + n] = p.detach().numpy()
    for n, g in zip(names, grads[:-1]):
        arrays["grad." + n] = g.numpy()
    # a second, independent check of the 9-step denoiser output and FM-returned x
    if not extras:
        arrays.update({"meta.B": np.array(B), "meta.T": np.array(T)})
        np.savez_compressed(out_path, **arrays)
        print("wrote", out_path, out_vals(arrays))
        return
    with torch.no_grad():
        z = heads.sproj(s.transpose(1, 2))
        proxy.queue.append(eps)
        zn, gamma = heads.adapter(z)
        zd = heads.denoiser(zn)
        fm, xo = heads.fm_latent(zd, heads.tae.enc(t.transpose(1, 2)))
    arrays.update({"out.gamma": gamma.numpy(), "out.z_deno": zd.numpy(), "out.fm_x": xo.numpy(),
                   "meta.B": np.array(B), "meta.T": np.array(T)})
    np.savez_compressed(out_path, **arrays)
    print("wrote", out_path, out_vals(arrays))


def out_vals(arrays):
    return f"recon {float(arrays['out.recon']):.6f} fm {float(arrays['out.fm_post']):.6f}"


if __name__ == "__main__":
    main()
    main(B=1, T=401, seed=11, out_path=OUT.replace(".npz", "_b1t401.npz"), extras=False)
    sys.exit(0)
