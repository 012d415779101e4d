"""Micro-benchmark of the fused SimpleDenoiser chain kernels at the bench shape (16 layers x B=32
utterances x T'=401 frames, L=96, 9 steps) and of its two CONV weight-gradient launches.
usage: python tools/deno_micro.py [reps]   (prints average µs per launch)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))


def main():
    from kdfm import kernels as K
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    T, U, L, S = 401, 16 * 32, 96, 9
    n = T * U
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    z = torch.randn(n, L, device=dev, generator=g)
    W1 = torch.randn(L, L, 3, device=dev, generator=g) * 0.05
    W2 = torch.randn(L, L, 3, device=dev, generator=g) * 0.05
    b1 = torch.zeros(L, device=dev)
    b2 = torch.zeros(L, device=dev)
    X = torch.empty(S, n, L, device=dev, dtype=torch.bfloat16)
    A = torch.empty_like(X)
    GV = torch.empty_like(X)
    DA = torch.empty_like(X)
    out = torch.empty(n, L, device=dev)
    gin = torch.empty(n, L, device=dev)
    g1 = torch.zeros(L, 3 * L, device=dev)
    db = torch.zeros(L, device=dev)

    def fwd():
        K.denoise_chain_fwd(z, W1, b1, W2, b2, X, A, out, T, S)

    def bwd():
        K.denoise_chain_bwd(out, A, W1, W2, GV, DA, gin, T, S)

    def wgr():
        K.wgrad_bf16_conv(DA.view(S * n, L), X.view(S * n, L), g1, T, db=db)

    for name, fn in (("denoise_fwd", fwd), ("denoise_bwd", bwd), ("wgrad_bf16_conv", wgr)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        print(f"{name:18s} {us:9.1f} us", flush=True)
    time.sleep(0.1)


if __name__ == "__main__":
    main()
