"""Micro-benchmark of the depthwise k=31 conv kernels at the bench shapes (B=32 utterances x T=401
frames, student d=88 / teacher d=176): forward with and without the fused BatchNorm statistics, and
the backward.  usage: python tools/dwconv_micro.py [reps]   (prints average us per launch)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))


def main():
    from kdfm import kernels as K
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    B, T, k = 32, 401, 31
    dev = "cuda"
    for d in (88, 176):
        gen = torch.Generator(device=dev).manual_seed(0)
        g = torch.randn(B * T, d, device=dev, generator=gen)
        w = torch.randn(d, k, device=dev, generator=gen) * 0.1
        bias = torch.zeros(d, device=dev)
        y = torch.empty_like(g)
        dg = torch.empty_like(g)
        dw = torch.zeros(d, k, device=dev)
        db = torch.zeros(d, device=dev)
        stats = torch.zeros(2 * d, device=dev, dtype=torch.float64)

        def fwd_stats():
            K.dwconv_fwd(g, w, bias, y, stats, B, T, d, k)

        def fwd_plain():
            K.dwconv_fwd(g, w, bias, y, None, B, T, d, k)

        def bwd():
            K.dwconv_bwd(y, g, w, dg, dw, db, B, T, d, k)

        mean, rstd = torch.zeros(d, device=dev), torch.ones(d, device=dev)
        gm, bt = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        red = torch.zeros(2 * d, dtype=torch.float64, device=dev)
        red_next = torch.zeros_like(red)
        dgm, dbt = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
        ws = torch.empty(K.dwconv_bwd_ws(B, T, d, k), device=dev)

        def bwd_bn():   # the step's form: BN-SiLU backward applied on load, partials left for the fold
            K.dwconv_bwd_bn(y, g, mean, rstd, gm, bt, red, red_next, dgm, dbt, True, g, w, dg, ws, B, T, d, k)

        cases = []
        for flag in ("0", "2", "0", "2"):   # KDFM_DWC_P2: 0 one channel per lane, 2 channel pairs
            cases += [(f"fwd+stats p2={flag}", fwd_stats, flag), (f"fwd p2={flag}", fwd_plain, flag),
                      (f"bwd p2={flag}", bwd, flag), (f"bwd_bn p2={flag}", bwd_bn, flag)]
        for case in cases:
            name, fn = case[0], case[1]
            if len(case) > 2:
                os.environ["KDFM_DWC_P2"] = case[2]
            fn()
            torch.cuda.synchronize()
            # a captured graph of reps calls: GPU time without the host's per-call issue
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(reps):
                    fn()
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            print(f"d={d:3d} {name:16s} {us:9.1f} us", flush=True)
    time.sleep(0.1)


if __name__ == "__main__":
    main()
