"""Which host calls of one training step take long on the host (a blocking runtime call shows up
as a multi-ms ctypes or torch call)?  Wraps kdfm.kernels.call and torch allocation/copy entry points."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402

dev = torch.device("cuda", 0)
K.set_math(DEFAULT.math)
eng = Ver5Engine(DEFAULT, dev)
wav, wl, tg, tl = synthetic_batch(DEFAULT, 32, 256000, 100, dev, seed=1234)
for _ in range(3):
    eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()

log = []
orig = K.call


def timed(name, *a):
    t0 = time.perf_counter()
    r = orig(name, *a)
    log.append((time.perf_counter() - t0, name, t0))
    return r


K.call = timed
orig_empty = torch.empty


def empty(*a, **k):
    t0 = time.perf_counter()
    r = orig_empty(*a, **k)
    log.append((time.perf_counter() - t0, "torch.empty", t0))
    return r


torch.empty = empty
T0 = time.perf_counter()
eng.train_step(wav, wl, tg, tl, None)
T1 = time.perf_counter()
torch.cuda.synchronize()
T2 = time.perf_counter()
print(f"step host {1e3 * (T1 - T0):.2f} ms, +drain {1e3 * (T2 - T0):.2f} ms, {len(log)} timed calls, "
      f"sum {1e3 * sum(x[0] for x in log):.2f} ms", flush=True)
for d, n, t in sorted(log, reverse=True)[:15]:
    print(f"  {1e3 * d:8.3f} ms at +{1e3 * (t - T0):8.2f} ms  {n}", flush=True)
