"""Isolated timing of the MX quantisation (kdfm_fp8_quant_mx) at the XL activation shapes (6432 rows x 1024 / 4096
bf16 columns) and of the f32 -> bf16 cast (kdfm_cast_bf16_2d): us per launch and GB/s over the bytes moved."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kd-via-fm-in-asr_amd"))
import kdfm  # noqa: E402,F401
import torch  # noqa: E402
from kdfm import kernels as K  # noqa: E402


def bench(fn, n=50, rounds=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3 / n)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    for cols in (1024, 4096):
        x16 = torch.randn(6432, cols, device=dev).bfloat16()
        x32 = torch.randn(6432, cols, device=dev)
        t = bench(lambda: K._fp8_operands([(x16, False)]))
        nb = x16.numel() * (2 + 1 + 1 / 32)
        print(f"quant bf16 6432x{cols}: {t * 1e6:7.1f} us  {nb / t / 1e9:7.1f} GB/s", flush=True)
        t = bench(lambda: K._fp8_operands([(x32, False)]))
        nb = x32.numel() * (4 + 1 + 1 / 32)
        print(f"quant f32  6432x{cols}: {t * 1e6:7.1f} us  {nb / t / 1e9:7.1f} GB/s", flush=True)
        t = bench(lambda: K._bf16_operands((x32,)))
        nb = x32.numel() * 6
        print(f"cast f32->bf16 6432x{cols}: {t * 1e6:7.1f} us  {nb / t / 1e9:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
