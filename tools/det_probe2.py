"""Probe: which gradients differ between two identical deterministic-mode engine runs."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kd-via-fm-in-asr_amd"))
from dataclasses import replace
import torch
from kdfm.config import DEFAULT
from kdfm.engine import Ver5Engine
from kdfm.overlap import WGRAD

if len(sys.argv) > 1 and sys.argv[1] == "nowgrad":
    WGRAD.enabled = False
cfg = replace(DEFAULT, n_layers=16, deterministic=True)
g = torch.Generator().manual_seed(21)
B, N = 4, 256000
wav = (0.1 * torch.randn(B, N, generator=g)).cuda()
wl = torch.tensor([256000, 256000, 230000, 256000], dtype=torch.int64).cuda()
tg = torch.randint(0, 128, (B, 60), generator=g).cuda()
tl = torch.full((B,), 60, dtype=torch.int64).cuda()
res = []
for _ in range(2):
    eng = Ver5Engine(cfg, "cuda")
    eng.set_seed(77)
    eng.advance_rng()
    ctx = eng.forward(wav, wl, tg, tl, train=True)
    eng.backward(ctx)
    torch.cuda.synchronize()
    res.append(eng.student.grads())
bad = [k for k in res[0] if not torch.equal(res[0][k], res[1][k])]
print("differing:", len(bad), "of", len(res[0]))
order = list(res[0].keys())
heads = [k for k in bad if not k.startswith(("encoder.", "decoder."))]
print("heads:", heads)
print("decoder:", [k for k in bad if k.startswith("decoder.")])
enc = [k for k in bad if k.startswith("encoder.")]
print("encoder (last 12):", enc[-12:])
