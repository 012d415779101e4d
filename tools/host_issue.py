"""Is the eager ver5 step host-issue bound?  Times (a) the Python/ctypes enqueue of one step (call
returns, no sync) and (b) the full step (enqueue + drain), for the bench configuration.
usage: python tools/host_issue.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
K.set_math(DEFAULT.math)
eng = Ver5Engine(DEFAULT, dev)
wav, wl, tg, tl = synthetic_batch(DEFAULT, 32, 256000, 100, dev, seed=1234)
for _ in range(3):
    eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()
enq, full = [], []
for _ in range(steps):
    t0 = time.perf_counter()
    eng.train_step(wav, wl, tg, tl, None)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enq.append(t1 - t0)
    full.append(t2 - t0)
print(f"enqueue {1e3 * min(enq):.2f} ms (median {1e3 * sorted(enq)[len(enq) // 2]:.2f}), "
      f"enqueue+drain {1e3 * min(full):.2f} ms (median {1e3 * sorted(full)[len(full) // 2]:.2f})", flush=True)
t0 = time.perf_counter()
for _ in range(steps):
    eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()
print(f"back-to-back {1e3 * (time.perf_counter() - t0) / steps:.2f} ms/step", flush=True)
# forward phase alone: host enqueue vs enqueue + drain
fe, ff = [], []
for _ in range(steps):
    eng.advance_rng()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx = eng.forward(wav, wl, tg, tl, train=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    fe.append(t1 - t0)
    ff.append(t2 - t0)
    eng.backward(ctx)
    del ctx
    torch.cuda.synchronize()
print(f"forward: enqueue {1e3 * min(fe):.2f} ms, enqueue+drain {1e3 * min(ff):.2f} ms", flush=True)
# the same step replayed from a recorded step plan (kdfm/plan.py): host enqueue vs enqueue + drain
plan = eng.make_plan(wav, wl, tg, tl)
torch.cuda.synchronize()
pe, pf = [], []
for _ in range(steps):
    t0 = time.perf_counter()
    plan.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    pe.append(t1 - t0)
    pf.append(t2 - t0)
print(f"step plan ({len(plan)} ops): enqueue {1e3 * min(pe):.2f} ms (median {1e3 * sorted(pe)[len(pe) // 2]:.2f}), "
      f"enqueue+drain {1e3 * min(pf):.2f} ms", flush=True)
t0 = time.perf_counter()
for _ in range(steps):
    plan.replay()
torch.cuda.synchronize()
print(f"step plan back-to-back {1e3 * (time.perf_counter() - t0) / steps:.2f} ms/step", flush=True)
