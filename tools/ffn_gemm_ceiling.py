"""How fast do library bf16 GEMMs (torch.matmul -> hipBLASLt) run the FFN's two products at the bench
shapes?  The ceiling a two-GEMM FFN (hidden through HBM) could reach, against the fused ffn_fwd kernels
(hidden kept on chip).  Times with HIP events over 50 reps after warmup."""
import torch

dev = torch.device("cuda", 0)
rows = 12832
for name, d in (("student", 176), ("teacher", 352)):
    h = 4 * d
    x = torch.randn(rows, d, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(d, h, device=dev, dtype=torch.bfloat16)
    w2 = torch.randn(h, d, device=dev, dtype=torch.bfloat16)
    hid = torch.randn(rows, h, device=dev, dtype=torch.bfloat16)
    for tag, fn in (("x@W1", lambda: x @ w1), ("h@W2", lambda: hid @ w2),
                    ("silu(x@W1)@W2", lambda: torch.nn.functional.silu(x @ w1) @ w2)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            fn()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 50 * 1e3
        fl = 2 * rows * d * h * (2 if "@W2" in tag and "silu" in tag else 1)
        print(f"{name:8s} {tag:14s} {us:7.1f} us  {fl / us / 1e6:7.1f} TFLOP/s")
