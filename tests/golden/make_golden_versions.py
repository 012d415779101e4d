"""Golden vectors for KD versions 1-8 (and kd_loss_type "l1") FROM THE REFERENCE'S OWN CODE.

Same extraction as make_golden.py (AST-selected class/function definitions of
/root/reference/asr_train_diffm.py exec'd with {torch, nn, F}; NoiseAdapter noise injected), now
driving `_compute_v_losses_one_layer` (asr_train_diffm.py:645-729) for every `version`.  Only numbers
are written (kd_heads_versions.npz): shared inputs/parameters, and per case the five loss terms,
d(total)/d(s) in full, and per-parameter gradient checksums (sum and sum of squares).

Usage:  python tests/golden/make_golden_versions.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import load_reference  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kd_heads_versions.npz")
KEYS = ("recon_loss", "kd_loss_pre", "fm_loss_pre", "kd_loss_post", "fm_loss_post")
CASES = [(v, "mse") for v in range(1, 9)] + [(1, "l1"), (3, "l1"), (8, "l1")]


def main(B=2, T=23, seed=11):
    ns, proxy = load_reference()
    Cs, Ct, L = 88, 176, 96
    flow_cfg = {"meta_encoder_type": "mlp", "feature_dim": Cs, "time_embed_dim": 32, "hidden_dim": L,
                "training_sampling": 8, "inference_sampling": 8, "weight": 1.0, "noise_schedule": "rectified",
                "loss": "mse", "shape_transform": "linear", "student_dim": Cs, "teacher_dim": Ct,
                "student_head_num": 2, "teacher_head_num": 4}

    class Heads(nn.Module):   # attributes of DistilFlowMatchingCTCModelBPE.__init__ (:553-564)
        def __init__(self, version, kd):
            super().__init__()
            self.version = version
            self.recon_crit = nn.MSELoss()
            self.kd_crit = nn.L1Loss() if kd == "l1" else nn.MSELoss()
            self.tae = ns["TeacherAutoEncoder"](teacher_dim=Ct, latent_dim=L)
            self.sproj = ns["StudentProjector"](student_dim=Cs, latent_dim=L)
            self.adapter = ns["NoiseAdapter"](latent_dim=L)
            self.denoiser = ns["SimpleDenoiser"](latent_dim=L, steps=9)
            self.fm_latent = ns["FMLatent"](latent_dim=L, flow_cfg=flow_cfg)
            self.fm_latent_2 = ns["FMLatent"](latent_dim=L, flow_cfg=flow_cfg)

    Heads._BHT_to_BTH = staticmethod(ns["_BHT_to_BTH"])
    Heads._compute_v_losses_one_layer = ns["_compute_v_losses_one_layer"]
    torch.manual_seed(seed)
    base = Heads(5, "mse")
    sd = {k: v.clone() for k, v in base.state_dict().items()}
    s0 = torch.randn(B, T, Cs)
    t = torch.randn(B, T, Ct)
    eps = torch.randn(B, L, T)
    arrays = {"in.s": s0.numpy(), "in.t": t.numpy(), "in.eps": eps.numpy(), "meta.B": np.array(B), "meta.T": np.array(T)}
    for k, v in sd.items():
        arrays["param." + k] = v.numpy()
    for version, kd in CASES:
        h = Heads(version, kd).train()
        h.load_state_dict(sd)
        s = s0.clone().requires_grad_(True)
        proxy.queue[:] = [eps]
        out = h._compute_v_losses_one_layer(s, t)
        total = sum(out[k] for k in KEYS)
        params = dict(h.named_parameters())
        names = list(params)
        grads = torch.autograd.grad(total, [params[n] for n in names] + [s], allow_unused=True)
        tag = f"v{version}{kd}"
        for k in KEYS:
            arrays[f"{tag}.{k}"] = np.array(float(out[k]), dtype=np.float64)
        arrays[f"{tag}.grad.s"] = grads[-1].numpy()
        for n, g in zip(names, grads[:-1]):
            g = torch.zeros_like(params[n]) if g is None else g
            arrays[f"{tag}.gsum.{n}"] = np.array([float(g.double().sum()), float((g.double() ** 2).sum())])
        print(tag, {k: round(float(out[k]), 6) for k in KEYS})
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
