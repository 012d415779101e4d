"""Isolated timing of the prepared-operand attention forward (kv prep + fwd3) at the bench's student (H 2,
d 88) and teacher (H 4, d 176) shapes, B 32 x T 401, with and without attention dropout, and both shapes
launched together on two streams (the step's overlap).  usage: python tools/attn3_micro.py [--pmc]  (--pmc: only the teacher shape with dropout, a few launches,
for rocprofv3 --pmc passes)"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402


def bench(name, fn, reps=30):
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


PMC = "--pmc" in sys.argv
g = torch.Generator(device="cuda").manual_seed(0)
B, T = 32, 401
seed = torch.tensor([1], dtype=torch.int64, device="cuda")
cases = {}
for (H, d) in (((4, 176),) if PMC else ((2, 88), (4, 176))):
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device="cuda", generator=g)
    qu = torch.randn(rows, d, device="cuda", generator=g)
    qv = torch.randn(rows, d, device="cuda", generator=g)
    ppos = torch.randn(2 * T - 1, d, device="cuda", generator=g)
    lens = torch.full((B,), T, dtype=torch.int64, device="cuda")
    o = torch.empty(rows, d, device="cuda")
    lse = torch.empty(B, H, T, device="cuda")
    sc = 1.0 / math.sqrt(d // H)
    prep = K.attn_kv_prep(qkv, lens, B, H, T)
    pb = K.attn_band_prep(ppos, H, T)[0]
    cases[H] = (qu, qv, prep, pb, lens, o, lse, sc, d, qkv)
    if PMC:
        for _ in range(4):
            K.relpos_attn_fwd3(qu, qv, prep, pb, lens, o, B, H, T, sc, 0.1, seed, 5, lse=lse)
        torch.cuda.synchronize()
        sys.exit(0)
    bench(f"H={H} kv prep", lambda: K.attn_kv_prep(qkv, lens, B, H, T))
    for p in (0.0, 0.1):
        bench(f"H={H} fwd3 p={p}", lambda: K.relpos_attn_fwd3(qu, qv, prep, pb, lens, o, B, H, T, sc, p, seed, 5,
                                                              lse=lse))
s2 = torch.cuda.Stream()


def both(p):
    a = cases[2]
    K.relpos_attn_fwd3(a[0], a[1], a[2], a[3], a[4], a[5], B, 2, T, a[7], p, seed, 5, lse=a[6])
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
        c = cases[4]
        K.relpos_attn_fwd3(c[0], c[1], c[2], c[3], c[4], c[5], B, 4, T, c[7], p, seed, 5, lse=c[6])
    torch.cuda.current_stream().wait_stream(s2)


for p in (0.0, 0.1):
    bench(f"student + teacher on two streams p={p}", lambda: both(p))
