"""Micro-benchmark of the weight-gradient products (linear_dw / conv3_dw, bf16) at the bench shapes:
average time per call with HIP events and algorithmic GB/s (dY and X read once, dW written once)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kd-via-fm-in-asr_amd"))
import torch
from kdfm import kernels as K

K.set_math("bf16")
if os.environ.get("DET"):
    K.set_deterministic(True)
dev = "cuda"
torch.manual_seed(0)
cases = [("ffn W2", 12832, 88, 352, False), ("ffn W1", 12832, 352, 88, False), ("qkv", 12832, 264, 88, False),
         ("pw1", 12832, 176, 88, False), ("out", 12832, 88, 88, False), ("sub out", 12832, 88, 1760, False),
         ("heads 96x96", 205312, 96, 96, False), ("tae.enc", 205312, 96, 176, False),
         ("tae.dec", 205312, 176, 96, False), ("deno conv3", 205312, 96, 96, True)]
for name, R, M, Kd, conv in cases:
    dy = torch.randn(R, M, device=dev)
    x = torch.randn(R, Kd, device=dev)
    if conv:
        G = torch.zeros(M, 3 * Kd, device=dev)
    else:
        G = torch.zeros(M, Kd, device=dev)
    db = torch.zeros(M, device=dev) if name != "sub out" else None
    def run():
        if conv:
            K.conv3_dw(dy, x, G, 401, db=db)
        else:
            K.linear_dw(dy, x, G, db=db)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    # replay a captured graph of n calls: GPU time without the Python launch overhead
    n = 20
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            run()
    gr.replay()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    nbytes = 4.0 * (R * M + R * Kd + M * (G.shape[1] + 1))
    print(f"{name:12s} R={R:6d} M={M:3d} N={G.shape[1]:4d}  {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s  route={K.ROUTES.get(int(K._lib.lib().kdfm_gemm_last_route()))}")

# bf16 row operands (kdfm_wgrad_bf16 / _conv: the fused kernels' saved operands), bytes at 2 B/element
bcases = [("ffn W2", 12832, 88, 352), ("ffn W1", 12832, 352, 88), ("qkv", 12832, 264, 88), ("out", 12832, 88, 88),
          ("fm dW1x", 205312, 96, 96), ("fm dW2", 8 * 205312, 96, 96), ("deno conv3", 9 * 205312, 96, 96)]
for name, R, M, N in bcases:
    conv = name.startswith("deno")
    dy = torch.randn(R, M, device=dev).to(torch.bfloat16)
    x = torch.randn(R, N, device=dev).to(torch.bfloat16)
    G = torch.zeros(M, 3 * N if conv else N, device=dev)
    db = torch.zeros(M, device=dev)
    def run():
        if conv:
            K.wgrad_bf16_conv(dy, x, G, 401, db=db)
        else:
            K.wgrad_bf16(dy, x, G, db=db)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    n = 10
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(n):
            run()
    gr.replay()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    nbytes = 2.0 * R * (M + N) + 8.0 * M * (G.shape[1] + 1)
    print(f"bf16 {name:10s} R={R:7d} M={M:3d} N={G.shape[1]:4d}  {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s", flush=True)
    del dy, x

# the FM chain's dW1x over its 8 steps: 8 per-step launches vs one segmented launch
R, M, S8 = 205312, 96, 8
dy = torch.randn(S8 * R, M, device=dev).to(torch.bfloat16)
x = torch.randn(S8 * R, M, device=dev).to(torch.bfloat16)
G = torch.zeros(M, M, device=dev)
dc = torch.zeros(S8, M, device=dev)
for name, run in (("8 launches", lambda: [K.wgrad_bf16(dy[j * R:(j + 1) * R], x[j * R:(j + 1) * R], G, db=dc[j])
                                          for j in range(S8)]),
                  ("segmented", lambda: K.wgrad_bf16_seg(dy, x, G, dc, R))):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    print(f"fm dW1x x8 {name:10s} {us:8.1f} us  {2.0 * S8 * R * 2 * M / us / 1e3:7.1f} GB/s", flush=True)
