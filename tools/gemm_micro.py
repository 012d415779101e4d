"""Micro-benchmark of the step's dominant GEMM shapes (bf16 math), each timed with HIP events over
20 launches after 3 warm-ups; prints us/launch, algorithmic TFLOP/s and unique-byte GB/s.
usage: python tools/gemm_micro.py [filter-substring]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402

flt = sys.argv[1] if len(sys.argv) > 1 else ""
dev = "cuda"
K.set_math("bf16")
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s):
    return torch.randn(*s, device=dev, generator=g)


def bench(name, fn, flops, nbytes, reps=20):
    if flt and flt not in name:
        return
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
    us = s.elapsed_time(e) / reps * 1e3
    print(f"{name:46s} {us:9.1f} us  {flops / us / 1e6:8.1f} TFLOP/s  {nbytes / us / 1e3:8.1f} GB/s", flush=True)


n, L, T = 205312, 96, 401
x = rnd(n, L)
y = torch.empty(n, L, device=dev)
R = rnd(n, L)
W = rnd(L, L) * 0.1
b = rnd(L)
Wf = rnd(L, 3 * L) * 0.05
bench("heads linear 205312x96x96 relu", lambda: K.linear(x, W, b, y, epi=_lib.EPI_RELU), 2 * n * L * L, 8 * n * L)
bench("heads linear 205312x96x96 resid", lambda: K.linear(x, W, b, y, epi=_lib.EPI_RESID, R=R, rscale=-0.125),
      2 * n * L * L, 12 * n * L)
bench("heads conv3 205312x96x288 relu", lambda: K.conv3(x, Wf, b, y, T, epi=_lib.EPI_RELU), 2 * n * L * 3 * L,
      8 * n * L)
G = torch.zeros(L, 3 * L, device=dev)
db = torch.zeros(L, device=dev)
bench("heads conv3_dw 96x289x205312", lambda: K.conv3_dw(R, x, G, T, db=db), 2 * n * L * (3 * L + 1), 8 * n * L)
dW = torch.zeros(L, L, device=dev)
bench("heads linear_dw 96x97x205312", lambda: K.linear_dw(R, x, dW, db=db), 2 * n * L * (L + 1), 8 * n * L)
m = 12832
xe = rnd(m, 88)
he = rnd(m, 352)
W1 = torch.zeros(352, 88, device=dev)
b1 = torch.zeros(352, device=dev)
bench("enc linear_dw 352x89x12832", lambda: K.linear_dw(he, xe, W1, db=b1), 2 * m * 352 * 89, 4 * m * (352 + 88))
W2 = torch.zeros(88, 352, device=dev)
b2 = torch.zeros(88, device=dev)
bench("enc linear_dw 88x353x12832", lambda: K.linear_dw(xe, he, W2, db=b2), 2 * m * 352 * 89, 4 * m * (352 + 88))
Wt = rnd(704, 176) * 0.1
xt = rnd(m, 176)
ht = torch.empty(m, 704, device=dev)
bench("enc linear 12832x704x176 silu", lambda: K.linear(xt, Wt, None, ht, epi=_lib.EPI_SILU), 2 * m * 704 * 176,
      4 * m * (704 + 176))
