"""Micro-benchmark of the striding subsampling's conv2 weight gradient gathered from the bf16 y1
(kdfm_wgrad_bf16_s2conv) at the bench shape (B=32, y1 801 x 40 x 88), plain vs XCD-grouped dispatch order
of its 3 column slices (KDFM_WGR_XGRP), plus a multi-slice linear product; average us per call over a
captured graph.  usage: python tools/s2conv_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))


def timed(run, n=10):
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            run()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    from kdfm import kernels as K
    B, T1, F1, C = 32, 801, 40, 88
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    X = torch.randn(B * T1 * F1, C, device="cuda").bfloat16()
    dY = torch.randn(B * T2 * F2, C, device="cuda").bfloat16()
    lin = torch.full((B,), T1, dtype=torch.int64, device="cuda")
    dW, db = torch.zeros(C, 9 * C, device="cuda"), torch.zeros(C, device="cuda")
    R, M, N = 12832, 88, 1760
    dy = torch.randn(R, M, device="cuda").bfloat16()
    x = torch.randn(R, N, device="cuda").bfloat16()
    G = torch.zeros(M, N, device="cuda")
    for rep in range(2):
        for flag in ("0", "1"):
            os.environ["KDFM_WGR_XGRP"] = flag
            us = timed(lambda: K.wgrad_bf16_s2conv(dY, X, lin, dW, db, B, T1, F1, C))
            nb = 2.0 * (X.numel() + dY.numel())
            us2 = timed(lambda: K.wgrad_bf16(dy, x, G))
            print(f"rep {rep} XGRP={flag}: s2conv {us:8.1f} us ({nb / us / 1e3:7.1f} GB/s operands)   "
                  f"linear {R}x{M}x{N} {us2:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
