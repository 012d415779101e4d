"""Cost of a cross-stream link event per kernel boundary: a chain of N small kernels on stream A, after each
an event recorded on A that stream B waits for (B runs a tiny kernel after each wait, as the weight-gradient
stream does), with the event created as torch.cuda.Event (HIP's default system-scope release fence), with
hipEventReleaseToDevice, with hipEventDisableSystemFence, and with no events at all.  HIP events around the
chain on A, median of 5 reps.  usage: python tools/event_micro.py"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
A, Bs = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
x = torch.ones(1 << 22, device=dev)
y = torch.ones(1 << 10, device=dev)
N = 200


def chain(kind):
    evs = None
    if kind == "system":
        evs = [torch.cuda.Event() for _ in range(4)]
    elif kind in ("device", "nofence"):
        evs = [K.LinkEvent({"device": 0x40000000, "nofence": 0x20000000}[kind]) for _ in range(4)]
    with torch.cuda.stream(A):
        for i in range(N):
            x.mul_(1.0000001)
            if evs is not None:
                ev = evs[i % 4]
                ev.record(A)
                ev.wait(Bs)
                with torch.cuda.stream(Bs):
                    y.add_(1.0)


def timed(kind, reps=5):
    out = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(A)
        chain(kind)
        b.record(A)
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / N)
    return statistics.median(out[1:])


for kind in ("none", "system", "device", "nofence", "none", "system", "device", "nofence"):
    print(f"{kind:8s} {timed(kind):7.2f} us per kernel on A (chain of {N})")
