"""Probe: which saved forward tensors differ between identical deterministic-mode forwards."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kd-via-fm-in-asr_amd"))
from dataclasses import replace
import torch
from kdfm.config import DEFAULT
from kdfm.engine import Ver5Engine


def flat(ctx):
    out = {}
    def walk(pref, o):
        if isinstance(o, torch.Tensor):
            out[pref] = o.detach().clone()
        elif isinstance(o, dict):
            for k, v in o.items():
                walk(f"{pref}.{k}", v)
        elif isinstance(o, (list, tuple)):
            for i, v in enumerate(o):
                walk(f"{pref}[{i}]", v)
        elif hasattr(o, "__dict__") and not isinstance(o, (int, float, str)):
            for k, v in vars(o).items():
                walk(f"{pref}.{k}", v)
    walk("ctx", ctx)
    return out


cfg = replace(DEFAULT, n_layers=16, deterministic=True)
g = torch.Generator().manual_seed(21)
B, N = 4, 256000
wav = (0.1 * torch.randn(B, N, generator=g)).cuda()
wl = torch.tensor([256000, 256000, 230000, 256000], dtype=torch.int64).cuda()
tg = torch.randint(0, 128, (B, 60), generator=g).cuda()
tl = torch.full((B,), 60, dtype=torch.int64).cuda()
eng = Ver5Engine(cfg, "cuda")
ref = None
for it in range(6):
    eng.set_seed(77)
    eng.advance_rng()
    ctx = eng.forward(wav, wl, tg, tl, train=True)
    torch.cuda.synchronize()
    f = flat(ctx)
    if ref is None:
        ref = f
        print("tensors", len(f))
        continue
    bad = [k for k in ref if k in f and ref[k].shape == f[k].shape and not torch.equal(ref[k], f[k])]
    print(it, "differing:", len(bad), bad[:12])
