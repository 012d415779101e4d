"""Does a HIP graph replay block the host?  Captures a chain of ~8 ms of GPU work on a side stream and
times the host side of replay() against the GPU time, with and without a pending second stream."""
import time

import torch

dev = torch.device("cuda", 0)
side = torch.cuda.Stream(dev)
x = torch.randn(8192, 8192, device=dev)
y = torch.empty_like(x)
with torch.cuda.stream(side):
    torch.mm(x, x, out=y)      # library handles initialised outside the capture
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    for _ in range(20):
        torch.mm(x, x, out=y)
torch.cuda.synchronize()
for _ in range(3):
    with torch.cuda.stream(side):
        g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(side):
    g.replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"replay() host {1e3 * (t1 - t0):.3f} ms, GPU drain {1e3 * (t2 - t0):.3f} ms", flush=True)
# eager equivalent
t0 = time.perf_counter()
with torch.cuda.stream(side):
    for _ in range(20):
        torch.mm(x, x, out=y)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"eager host {1e3 * (t1 - t0):.3f} ms, GPU drain {1e3 * (t2 - t0):.3f} ms", flush=True)
print("driver version", torch.cuda.get_device_properties(0), flush=True)

# does work issued on the main stream right after a side-stream replay wait for the graph?
main = torch.cuda.current_stream(dev)
z = torch.randn(1024, device=dev)
torch.cuda.synchronize()
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
e0.record(main)
z.add_(1.0)
side.wait_stream(main)
with torch.cuda.stream(side):
    g.replay()
z.mul_(2.0)
e1.record(main)
torch.cuda.synchronize()
print(f"main-stream op after a side replay completed {e0.elapsed_time(e1):.3f} ms after the replay was issued", flush=True)
e0.record(main)
z.add_(1.0)
side.wait_stream(main)
with torch.cuda.stream(side):
    for _ in range(20):
        torch.mm(x, x, out=y)
z.mul_(2.0)
e1.record(main)
torch.cuda.synchronize()
print(f"main-stream op after eager side work completed {e0.elapsed_time(e1):.3f} ms", flush=True)

# the same with a created (non-null) stream as "main"
main2 = torch.cuda.Stream(dev)
with torch.cuda.stream(main2):
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(main2)
    z.add_(1.0)
    side.wait_stream(main2)
    with torch.cuda.stream(side):
        g.replay()
    z.mul_(2.0)
    e1.record(main2)
    torch.cuda.synchronize()
    print(f"[non-null main] op after a side replay completed {e0.elapsed_time(e1):.3f} ms after the replay was issued",
          flush=True)
