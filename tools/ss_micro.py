"""Isolated timing of the one-kernel striding subsampling forward (kdfm_subsample_fused) at the bench
shape (B = 32, 16 s: Tm = 1601 mel frames) for the student (C = 88, with the y1 side output) and the
teacher (C = 176), plus the two run concurrently on two streams as in the step.  HIP events, 20 reps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
B, Tm, F = 32, 1601, 80
T1, F1 = (Tm - 1) // 2 + 1, (F - 1) // 2 + 1
T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
g = torch.Generator(device=dev).manual_seed(0)
mel = torch.randn(B, Tm, F, device=dev, generator=g)
ml = torch.full((B,), Tm, dtype=torch.int64, device=dev)
l1 = torch.full((B,), T1, dtype=torch.int64, device=dev)
l2 = torch.full((B,), T2, dtype=torch.int64, device=dev)
runs = {}
for C, side in ((88, True), (176, False)):
    w0 = torch.randn(C, 1, 3, 3, device=dev, generator=g) * 0.3
    w2 = torch.randn(C, C, 3, 3, device=dev, generator=g) * (1.0 / (3 * C ** 0.5))
    b0 = torch.randn(C, device=dev, generator=g) * 0.1
    b2 = torch.randn(C, device=dev, generator=g) * 0.1
    wp = torch.empty(K.subsample_fused_wprep_elems(C), device=dev, dtype=torch.bfloat16)
    K.subsample_fused_wprep(w0, w2, wp)
    y2 = torch.empty(B * T2 * F2, C, device=dev)
    ld = int(os.environ.get("SS_Y1_LD", str(C)))   # y1 row stride (96: the step's padded rows)
    y1 = torch.empty(B * T1 * F1, ld, device=dev, dtype=torch.bfloat16) if side else None
    runs[C] = lambda wp=wp, b0=b0, b2=b2, y2=y2, y1=y1, C=C: K.subsample_fused(mel, ml, l1, l2, wp, b0, b2, y2, y1,
                                                                            B, Tm, F, C)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for C, fn in runs.items():
    flop = 2 * 9 * C * C * B * T2 * F2
    us = timed(fn)
    print(f"C={C:3d} isolated: {us:7.1f} us  conv2 {flop / us / 1e6:6.1f} TFLOP/s")
s2 = torch.cuda.Stream(dev)


def both():
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
        runs[176]()
    runs[88]()
    torch.cuda.current_stream().wait_stream(s2)


print(f"student + teacher on two streams: {timed(both):7.1f} us")

# the backward's direct conv2 data gradient with conv0's weight gradient fused (student, C = 88)
C = 88
w2 = torch.randn(C, C, 3, 3, device=dev, generator=g) * (1.0 / (3 * C ** 0.5))
wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device=dev, dtype=torch.bfloat16)
K.subsample_dgrad_wprep(w2, wt)
dy2 = torch.randn(B * T2 * F2, C, device=dev, generator=g)
y1 = torch.randn(B * T1 * F1, C, device=dev, generator=g).to(torch.bfloat16)
dw0 = torch.zeros(C, 9, device=dev)
db0 = torch.zeros(C, device=dev)
us = timed(lambda: K.subsample_conv2_dgrad_w0(dy2, wt, y1, B, T1, F1, C, mel, ml, Tm, F, 1, dw0, db0))
print(f"C={C:3d} conv2 dgrad + conv0 wgrad isolated: {us:7.1f} us  ({2 * 2.25 * C * C * B * T1 * F1 / us / 1e6:6.1f} TFLOP/s)")
