"""Micro-benchmark of the fused rel-pos attention forward (training: O + per-row lse) and backward kernels at
the student bench shape (B=32 utterances, H=2 heads, T'=401 frames, d=88, attention dropout 0.1).
usage: python tools/attn_bwd_micro.py [reps] [p_drop]   (run under rocprofv3 --kernel-trace --stats for
the per-kernel split)"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
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
    P = torch.empty(B, H, T, T, device=dev)
    lse, pt, mblk = K.attn_saved(B, H, T, dev)
    o = torch.empty(rows, d, device=dev)
    dqu = torch.empty(rows, d, device=dev)
    dqv = torch.empty_like(dqu)
    dqkv = torch.zeros(rows, 3 * d, device=dev)
    dpos = torch.empty(2 * T - 1, d, device=dev)
    sc = 1.0 / math.sqrt(dk)

    def fwd_p():
        K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, P, None, B, H, T, sc, p, seed, 11)

    def fwd_lse():
        K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, None, None, B, H, T, sc, p, seed, 11, lse=lse)

    def fwd():
        K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, None, None, B, H, T, sc, p, seed, 11, lse=lse, p_tilde=pt,
                          m_blk=mblk)

    def bwd():
        K.relpos_attn_bwd(do, o, qu, qv, qkv, ppos, lse, pt, mblk, lens, dqu, dqv, dqkv, dpos, B, H, T, sc, p, seed,
                          11)

    for name, fn in (("relpos_attn_fwd (two-pass, P)", fwd_p), ("relpos_attn_fwd (one pass, lse)", fwd_lse),
                     ("relpos_attn_fwd (one pass, lse + p~)", fwd), ("relpos_attn_bwd (all kernels)", bwd)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"{name:32s} {s.elapsed_time(e) / reps * 1e3:9.1f} us", flush=True)


if __name__ == "__main__":
    main()
