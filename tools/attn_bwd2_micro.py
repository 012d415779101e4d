"""Micro-benchmark of the attention backward v2 kernels (csrc/attn_bwd.hip bwd2: dQ + saved dS / Pd, dK / dV,
dPpos) at the student bench shape (B=32, H=2, T'=401, d=88, attention dropout 0.1): each alone, and the dQ
kernel while a weight-gradient burst (student FFN linear2 shape, 12832 x 352 -> 88) runs on a second stream,
as in the step's backward.  usage: python tools/attn_bwd2_micro.py [reps]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    p = 0.1
    B, H, T, d = 32, 2, 401, 88
    dk = d // H
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device=dev, generator=g)
    qu = torch.randn(rows, d, device=dev, generator=g)
    qv = torch.randn(rows, d, device=dev, generator=g)
    ppos = torch.randn(2 * T - 1, d, device=dev, generator=g)
    do = torch.randn(rows, d, device=dev, generator=g)
    lens = torch.full((B,), T, dtype=torch.int64, device=dev)
    lens[1::3] = T - 57
    seed = torch.tensor([7], dtype=torch.int64, device=dev)
    lse, _, _ = K.attn_saved(B, H, T, dev)
    o = torch.empty(rows, d, device=dev)
    dqu = torch.empty(rows, d, device=dev)
    dqv = torch.empty_like(dqu)
    dqkv = torch.zeros(rows, 3 * d, device=dev)
    dpos = torch.empty(2 * T - 1, d, device=dev)
    ds, pd = K.attn_bwd2_saved(B, H, T, dev)
    sc = 1.0 / math.sqrt(dk)
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, None, None, B, H, T, sc, p, seed, 11, lse=lse)

    def dq():
        K.relpos_attn_bwd2_dq(do, o, qu, qv, qkv, ppos, lse, lens, None, ds, pd, dqu, dqv, B, H, T, sc, p, seed, 11)

    def dkv():
        K.relpos_attn_bwd2_dkv(do, qu, ds, pd, lens, dqkv, B, H, T)

    def dp():
        K.relpos_attn_bwd2_dpos(qv, ds, lens, dpos, B, H, T)

    for name, fn in (("bwd2 dQ (+ dS / Pd)", dq), ("bwd2 dK / dV", dkv), ("bwd2 dPpos", dp)):
        print(f"{name:32s} {timed(fn, reps):9.1f} us", flush=True)

    # dQ beside a weight-gradient burst on a second stream
    dy = torch.randn(rows, d, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(rows, 4 * d, device=dev, generator=g).to(torch.bfloat16)
    dw = torch.zeros(d, 4 * d, device=dev)
    db = torch.zeros(d, device=dev)
    side = torch.cuda.Stream()
    tw = timed(lambda: K.wgrad_bf16(dy, x, dw, db=db), reps)
    print(f"{'wgrad 12832x88x352 alone':32s} {tw:9.1f} us", flush=True)
    for nw in (1, 2, 4):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(side):
                side.wait_event(ev)
                for _ in range(nw):
                    K.wgrad_bf16(dy, x, dw, db=db)
            dq()
            torch.cuda.current_stream().wait_stream(side)
        e.record()
        torch.cuda.synchronize()
        print(f"dQ + {nw} wgrad on a side stream    {s.elapsed_time(e) / reps * 1e3:9.1f} us (pair wall)", flush=True)


if __name__ == "__main__":
    main()
