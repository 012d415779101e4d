"""Where does the student subsampling conv2 data-gradient launch (ss_dgrad_kernel, ~650 us at the bench
shape) spend its time?  Times kdfm_subsample_conv2_dgrad (dy1 written, no conv0 weight gradient) against
kdfm_subsample_conv2_dgrad_w0 (conv0 weight gradient fused, dy1 not written, the training step's call)
at B=32, 16 s (T1=801, F1=40, C=88).
usage: python tools/ss_dgrad_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402

dev = torch.device("cuda")
B, Tm, Fm, C, pad = 32, 1601, 80, 88, 1
T1, F1 = (Tm + 2 * pad - 3) // 2 + 1, (Fm + 2 * pad - 3) // 2 + 1
T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
g = torch.Generator(device=dev).manual_seed(0)
dy2 = torch.randn(B * T2 * F2, C, device=dev, generator=g)
y1 = torch.randn(B * T1 * F1, C, device=dev, generator=g).to(torch.bfloat16)
mel = torch.randn(B, Tm, Fm, device=dev, generator=g)
mel_len = torch.full((B,), Tm, dtype=torch.int64, device=dev)
w2 = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.03
wt = torch.empty(K.subsample_dgrad_wprep_elems(C), dtype=torch.bfloat16, device=dev)
K.subsample_dgrad_wprep(w2, wt)
dy1 = torch.empty(B * T1 * F1, C, device=dev)
dw0 = torch.zeros(C, 9, device=dev)
db0 = torch.zeros(C, device=dev)


def timeit(label, fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{label:40s} {1e3 * s.elapsed_time(e) / n:8.1f} us", flush=True)


timeit("dgrad, dy1 written", lambda: K.subsample_conv2_dgrad(dy2, wt, y1, dy1, B, T1, F1, C))
timeit("dgrad_w0, dy1 not written (step call)",
       lambda: K.subsample_conv2_dgrad_w0(dy2, wt, y1, B, T1, F1, C, mel, mel_len, Tm, Fm, pad, dw0, db0))
timeit("dgrad_w0, no mel_len", lambda: K.subsample_conv2_dgrad_w0(dy2, wt, y1, B, T1, F1, C, mel, None, Tm, Fm, pad,
                                                                   dw0, db0))
timeit("dgrad_w0 + dy1", lambda: K.subsample_conv2_dgrad_w0(dy2, wt, y1, B, T1, F1, C, mel, mel_len, Tm, Fm, pad,
                                                             dw0, db0, dy1=dy1))
