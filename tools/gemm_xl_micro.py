"""Isolated timing of the FastConformer-XL layer products (d_model 1024, B=32 x 16 s at x8: 6 432 rows) -- the
routes the XL step takes at d=1024, where no fused LN-block kernel applies -- beside torch.matmul (hipBLASLt) on bf16
copies as the library yardstick.  Prints TFLOP/s per product and direction:
  big     : kernels.linear / linear_dx / linear_dw on the large-tile route (csrc/biggemm.hip) with bf16 operands in
            HBM (the kernel alone: what the XL step's bf16 intermediates feed it);
  big+cast: the same from f32 operands (each f32 operand cast to bf16 scratch first, kdfm_cast_bf16_2d);
  generic : the previous route (kdfm_gemm's 64x64 tile / row-parallel weight gradient), f32 operands;
  fp8+quant: the fp8 e4m3 instance (linear_fp8) including the MX quantisation of both operands;
  fp8 kernel: the fp8 kernel alone on operands quantised once.
HIP events around N back-to-back launches (median of 3 rounds)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kd-via-fm-in-asr_amd"))
import kdfm  # noqa: E402,F401
import torch  # noqa: E402
from kdfm import kernels as K  # noqa: E402


def bench(fn, n=20, rounds=3):
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
    K.set_math("bf16")
    M, d = 6432, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [("ffn_up", 4096, d), ("ffn_down", d, 4096), ("qkv", 3 * d, d), ("out", d, d)]
    if len(sys.argv) > 1 and sys.argv[1] == "large":   # Conformer-large (configs[3] student): d 512, 12 832 rows
        M, d = 12832, 512
        shapes = [("ffn_up", 2048, d), ("ffn_down", d, 2048), ("qkv", 3 * d, d), ("out", d, d)]
    for (name, N, Kd) in shapes:
        fl = 2.0 * M * N * Kd
        x = torch.randn(M, Kd, device=dev, generator=g)
        W = torch.randn(N, Kd, device=dev, generator=g) * 0.02
        b = torch.randn(N, device=dev, generator=g)
        dy = torch.randn(M, N, device=dev, generator=g)
        x16, dy16 = x.bfloat16(), dy.bfloat16()
        y = torch.empty(M, N, device=dev)
        dx = torch.empty(M, Kd, device=dev)
        dW = torch.zeros(N, Kd, device=dev)
        db = torch.zeros(N, device=dev)
        res = {}
        res["fwd big"] = bench(lambda: K.linear(x16, W, b, y))
        res["fwd big+cast"] = bench(lambda: K.linear(x, W, b, y))
        res["dx big"] = bench(lambda: K.linear_dx(dy16, W, dx))
        res["dx big+cast"] = bench(lambda: K.linear_dx(dy, W, dx))
        res["dW big"] = bench(lambda: K.linear_dw(dy16, x16, dW, db=db))
        res["dW big+cast"] = bench(lambda: K.linear_dw(dy, x, dW, db=db))
        K._State.fp8 = True
        try:
            res["fwd fp8+quant"] = bench(lambda: K.linear(x16, W, b, y))
            res["dx fp8+quant"] = bench(lambda: K.linear_dx(dy16, W, dx))
            # the fp8 kernel alone on operands quantised once (kernels._fp8_operands into a private copy)
            (a8, lda, sa), (w8, ldw, sw) = K._fp8_operands([(x16, False), (W, False)])
            q = K.scratch(dev, 1)
            keep = torch.empty(q.numel(), device=dev)
            keep.copy_(q)
            off = keep.data_ptr() - q.data_ptr()
            import kdfm._lib as L
            res["fwd fp8 kernel"] = bench(lambda: K.gemm(x16, W, y, M, N, Kd, 0, 0, 0, 0, y.stride(0), 1, amode=L.LD_KC,
                                                         bmode=L.LD_KC, epi=L.EPI_BIAS, bias=b,
                                                         fp8=(a8 + off, lda, w8 + off, ldw, sa + off, sw + off, 0)))
        finally:
            K._State.fp8 = False
        K._BIG = False
        try:
            res["fwd generic"] = bench(lambda: K.linear(x, W, b, y))
            res["dx generic"] = bench(lambda: K.linear_dx(dy, W, dx))
            res["dW generic"] = bench(lambda: K.linear_dw(dy, x, dW, db=db))
        finally:
            K._BIG = True
        Wb = W.bfloat16()
        res["fwd hipBLASLt"] = bench(lambda: torch.matmul(x16, Wb.t()))
        res["dx hipBLASLt"] = bench(lambda: torch.matmul(dy16, Wb))
        res["dW hipBLASLt"] = bench(lambda: torch.matmul(dy16.t(), x16))
        line = " | ".join(f"{k} {v * 1e6:7.1f} us {fl / v / 1e12:6.1f} TF/s" for k, v in res.items())
        print(f"{name:9s} M={M} N={N} K={Kd}: {line}", flush=True)


if __name__ == "__main__":
    main()
