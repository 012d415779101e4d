"""Micro-benchmark of the fused FM chain kernels at the bench shape (8 layers x 32 utterances x 401 frames =
102 656 latent rows, 96 features, 8 steps): forward (with the bf16 saves) and backward, average us per launch.
KDFM_LIB=ab/libkdfm_base.so runs a base library (tools/build_ab_base.sh) for a same-box A/B; the outputs of
both libraries are written to <out>.pt so they can be compared bit for bit.
usage: python tools/fmchain_micro.py [reps] [out.pt]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))


def main():
    from kdfm import kernels as K
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    out = sys.argv[2] if len(sys.argv) > 2 else None
    n, L, S = 8 * 32 * 401, 96, 8
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(n, L, device=dev, generator=g)
    zt = torch.randn(n, L, device=dev, generator=g)
    W1 = torch.randn(L, L + 32, device=dev, generator=g) * 0.1
    cvec = torch.randn(S, L, device=dev, generator=g) * 0.1
    W2 = torch.randn(L, L, device=dev, generator=g) * 0.1
    b2 = torch.randn(L, device=dev, generator=g) * 0.1
    Wst = torch.randn(L, L, device=dev, generator=g) * 0.1
    bst = torch.randn(L, device=dev, generator=g) * 0.1
    X = torch.empty(S, n, L, device=dev, dtype=torch.bfloat16)
    A = torch.empty_like(X)
    nsx, dtr, xS = torch.empty_like(x0), torch.empty_like(x0), torch.empty_like(x0)
    loss = torch.zeros(1, device=dev)
    DV, DA = torch.empty_like(X), torch.empty_like(X)
    gx0 = torch.empty_like(x0)

    def fwd():
        K.fm_chain_fwd(x0, zt, W1, cvec, W2, b2, Wst, bst, X, A, nsx, dtr, xS, loss, 1.0 / n, S)

    def bwd():
        K.fm_chain_bwd(dtr, A, xS, W1, W2, Wst, DV, DA, gx0, S)

    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"fm_chain {name}: {1e3 * e0.elapsed_time(e1) / reps:.1f} us", flush=True)
    if out:
        loss.zero_()
        fwd()
        bwd()
        torch.cuda.synchronize()
        torch.save({k: v.cpu() for k, v in dict(X=X, A=A, nsx=nsx, dtr=dtr, xS=xS, loss=loss, DV=DV, DA=DA,
                                                  gx0=gx0).items()}, out)


if __name__ == "__main__":
    main()
