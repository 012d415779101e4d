"""Micro-benchmark of the fused rel-pos attention forward vs the unfused bf16 path.
usage: python tools/attn_micro.py"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402
from test_attn_fused_gpu import _unfused  # noqa: E402


def bench(name, fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{name:50s} {s.elapsed_time(e) / reps * 1e3:9.1f} us", flush=True)


g = torch.Generator(device="cuda").manual_seed(0)
for (H, d) in ((4, 176), (2, 88)):
    B, T = 32, 401
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device="cuda", generator=g)
    qu = torch.randn(rows, d, device="cuda", generator=g)
    qv = torch.randn(rows, d, device="cuda", generator=g)
    ppos = torch.randn(2 * T - 1, d, device="cuda", generator=g)
    lens = torch.full((B,), T, dtype=torch.int64, device="cuda")
    seed = torch.tensor([1], dtype=torch.int64, device="cuda")
    o = torch.empty(rows, d, device="cuda")
    P = torch.empty(B, H, T, T, device="cuda")
    Pd = torch.empty(B, H, T, T, device="cuda")
    sc = 1.0 / math.sqrt(d // H)
    bench(f"H={H} fused, no P", lambda: K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, None, None, B, H, T, sc, 0.0,
                                                          None, 0))
    bench(f"H={H} fused, P", lambda: K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, P, None, B, H, T, sc, 0.0,
                                                       None, 0))
    bench(f"H={H} fused, P + Pd (dropout 0.1)",
          lambda: K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, P, Pd, B, H, T, sc, 0.1, seed, 5))
    bench(f"H={H} unfused (AC, BD, softmax, PV)",
          lambda: _unfused(K, _lib, qu, qv, qkv, ppos, lens, B, H, T, d, 0.1, seed))
