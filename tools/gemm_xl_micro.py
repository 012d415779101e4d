"""Isolated timing of the FastConformer-XL layer products (d_model 1024, B=32 x 16 s at x8: 6 432 rows) on
kdfm_gemm (bf16 math) -- the routes the XL step takes at d=1024, where no fused LN-block kernel applies --
beside torch.matmul (hipBLASLt) on bf16 copies as the library yardstick.  Prints TFLOP/s per product."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kd-via-fm-in-asr_amd"))
import kdfm  # noqa: E402,F401
import torch  # noqa: E402
from kdfm import kernels as K  # noqa: E402
from kdfm import _lib  # noqa: E402


def bench(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    dev = torch.device("cuda")
    K.set_math("bf16")
    M, d = 6432, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    for (name, N, Kd) in [("ffn_up", 4096, d), ("ffn_down", d, 4096), ("qkv", 3 * d, d), ("out", d, d)]:
        x = torch.randn(M, Kd, device=dev, generator=g)
        W = torch.randn(N, Kd, device=dev, generator=g) * 0.02
        b = torch.randn(N, device=dev, generator=g)
        y = torch.empty(M, N, device=dev)
        t = bench(lambda: K.linear(x, W, b, y))
        route = K.ROUTES.get(int(_lib.lib().kdfm_gemm_last_route()), "?")
        dy = torch.randn(M, N, device=dev, generator=g)
        dx = torch.empty(M, Kd, device=dev)
        tdx = bench(lambda: K.linear_dx(dy, W, dx))
        dW = torch.zeros(N, Kd, device=dev)
        tdw = bench(lambda: K.linear_dw(dy, x, dW))
        xb, Wb = x.bfloat16(), W.bfloat16()
        tl = bench(lambda: torch.matmul(xb, Wb.t()))
        fl = 2.0 * M * N * Kd
        print(f"{name:9s} M={M} N={N} K={Kd}: fwd {t * 1e6:8.1f} us {fl / t / 1e12:6.1f} TF/s ({route}) | dx "
              f"{tdx * 1e6:8.1f} us {fl / tdx / 1e12:6.1f} | dW {tdw * 1e6:8.1f} us {fl / tdw / 1e12:6.1f} | "
              f"hipBLASLt bf16 {tl * 1e6:8.1f} us {fl / tl / 1e12:6.1f}", flush=True)


if __name__ == "__main__":
    main()
