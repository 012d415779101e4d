"""Regenerates the inputs and parameters of tests/golden/kd_encfm_meta.npz without the reference
(make_golden_encfm_meta.py's seeded_params and input draws), for the oracle and engine tests."""
import ast
import os

import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_encfm_meta.npz")
SEED = 7


def load():
    return dict(np.load(GOLD, allow_pickle=False))


def params(z, meta, seed=SEED, dtype=torch.float32):
    """{name: tensor} in the fixture's named_parameters order: >= 2-D U(+-1/sqrt(fan_in)), 1-D '...weight'
    1 + 0.1 U, other 1-D 0.1 U, one CPU generator (seed * 1000 + index) per tensor."""
    out = {}
    for i, (n, shp) in enumerate(zip(z[meta + ".names"], z[meta + ".shapes"])):
        shape = tuple(ast.literal_eval(str(shp)))
        g = torch.Generator().manual_seed(seed * 1000 + i)
        u = torch.rand(shape, generator=g) * 2 - 1
        if len(shape) >= 2:
            p = u / (int(np.prod(shape[1:])) ** 0.5)
        elif str(n).endswith("weight"):
            p = 1.0 + 0.1 * u
        else:
            p = 0.1 * u
        out[str(n)] = p.to(dtype)
    return out


def inputs(z, seed=SEED, Cs=88, Ct=176, T=None):
    """(s list, t list, R) of (B, T, C) float32 tensors, drawn as the generator drew them (T: the unet entries'
    own frame count, "unet.meta.T")."""
    L, B = int(z["meta.L"]), int(z["meta.B"])
    T = int(z["meta.T"]) if T is None else int(T)
    gi = torch.Generator().manual_seed(seed + 99)
    s = [0.5 * torch.randn(B, T, Cs, generator=gi) for _ in range(L)]
    t = [torch.randn(B, T, Ct, generator=gi) for _ in range(L)]
    R = torch.randn(B, T, Cs, generator=gi)
    return s, t, R


def bn_init(z, meta):
    """BatchNorm running statistics at construction (mean 0, var 1), float64, named as the fixture's
    buffers (empty for meta-encoders without BatchNorm)."""
    out = {}
    pre = meta + ".buffer."
    for k in z:
        if k.startswith(pre) and k.endswith(("running_mean", "running_var")):
            name = k[len(pre):]
            shape = z[k].shape
            out[name] = torch.zeros(shape, dtype=torch.float64) if name.endswith("mean") else \
                torch.ones(shape, dtype=torch.float64)
    return out
