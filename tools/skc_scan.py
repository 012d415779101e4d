"""Scaling scan of the LDS-slab CONV kernel (denoiser Conv1d k=3, 96->96) against a plain device copy
of the same bytes: time vs rows tells fixed (weight staging, launch) from per-tile cost.
usage: python tools/skc_scan.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402

K.set_math("bf16")
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)


def timeit(fn, reps=20):
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


L, T = 96, 401
W = torch.randn(L, L, 3, device=dev, generator=g) * 0.05
wf, wb = torch.empty(L, 3 * L, device=dev), torch.empty(L, 3 * L, device=dev)
K.convw_prep(W, fwd=wf, bwd=wb)
b = torch.randn(L, device=dev, generator=g)
for n in (401 * 32, 401 * 128, 401 * 256, 205312, 401 * 1024, 401 * 2048):
    x = torch.randn(n, L, device=dev, generator=g)
    y = torch.empty(n, L, device=dev)
    R = torch.randn(n, L, device=dev, generator=g)
    us1 = timeit(lambda: K.conv3(x, wf, b, y, T, epi=_lib.EPI_RELU))
    us2 = timeit(lambda: K.conv3(x, wf, b, y, T, R=R, rscale=-1.0 / 9))
    usc = timeit(lambda: y.copy_(x))
    mb = n * L * 4 / 1e6
    print(f"rows {n:8d}  conv3 relu {us1:8.1f} us {2 * mb / us1 * 1e3:6.0f} GB/s | resid {us2:8.1f} us "
          f"{3 * mb / us2 * 1e3:6.0f} GB/s | copy {usc:7.1f} us {2 * mb / usc * 1e3:6.0f} GB/s", flush=True)
