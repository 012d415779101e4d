"""Golden vectors for the DiffKD head (use_diffkd) FROM THE REFERENCE'S OWN CLASS.

Same extraction as make_golden.py (AST-selected definitions of /root/reference/asr_train_diffm.py
exec'd with {torch, nn, F}), plus DiffKDModule (asr_train_diffm.py:326-394).  The reference's
training_step (:795-800) adds, when use_diffkd is set,
    diffkd_loss = (1 / L) * sum_l DiffKDModule(s_l, t_l),
    DiffKDModule(s, t) = MSE(dec(enc(t).detach()), t) + MSE(denoise^9(proj(s)), enc(t).detach())
over the L hooked layer pairs (s_l: (B, T, 88) student, t_l: (B, T, 176) teacher), with its own
encoder / decoder / proj / denoiser weights (diffkd_cfg: diffusion_steps, latent_dim = args.latent_dim,
:1830-1836).  Only numbers are written (kd_diffkd.npz): inputs, parameters, the loss, d(loss)/d(s_l)
in full and per-parameter gradients in full (the module is small).

Usage:  python tests/golden/make_golden_diffkd.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kd_diffkd.npz")


def main(L=3, B=2, T=23, steps=9, seed=13):
    make_golden.KEEP_CLASSES = set(make_golden.KEEP_CLASSES) | {"DiffKDModule"}
    ns, _ = make_golden.load_reference()
    Cs, Ct, Lt = 88, 176, 96
    torch.manual_seed(seed)
    mod = ns["DiffKDModule"]({"diffusion_steps": steps, "student_dim": Cs, "teacher_dim": Ct, "latent_dim": Lt})
    s = [torch.randn(B, T, Cs).requires_grad_(True) for _ in range(L)]
    t = [torch.randn(B, T, Ct) for _ in range(L)]
    loss = sum(mod(si, ti) for si, ti in zip(s, t)) / L
    params = dict(mod.named_parameters())
    names = list(params)
    # the encoder output is detached before both of its uses (:382-383): encoder.* get no gradient
    grads = torch.autograd.grad(loss, [params[n] for n in names] + s, allow_unused=True)
    arrays = {"meta.L": np.array(L), "meta.B": np.array(B), "meta.T": np.array(T), "meta.steps": np.array(steps),
              "loss": np.array(float(loss), dtype=np.float64)}
    for i in range(L):
        arrays[f"in.s{i}"] = s[i].detach().numpy()
        arrays[f"in.t{i}"] = t[i].numpy()
        arrays[f"grad.s{i}"] = grads[len(names) + i].numpy()
    for n, g in zip(names, grads[:len(names)]):
        arrays["param." + n] = params[n].detach().numpy()
        if g is not None:
            arrays["grad." + n] = g.numpy()
    np.savez_compressed(OUT, **arrays)
    print("diffkd loss", float(loss), "params", names, "untrained", [n for n, g in zip(names, grads) if g is None])
    print("wrote", OUT)


if __name__ == "__main__":
    main()
