"""Where does the host spend the enqueue of one eager training step?  cProfile of Ver5Engine.train_step
(no device sync inside the profiled region) at the bench configuration; prints the top functions by
own time and by cumulative time, plus the enqueue / enqueue+drain times.
usage: python tools/host_profile.py [top]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
K.set_math(DEFAULT.math)
eng = Ver5Engine(DEFAULT, dev)
wav, wl, tg, tl = synthetic_batch(DEFAULT, 32, 256000, 100, dev, seed=1234)
for _ in range(3):
    eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()
enq = []
for _ in range(5):
    t0 = time.perf_counter()
    eng.train_step(wav, wl, tg, tl, None)
    enq.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
print(f"enqueue median {1e3 * sorted(enq)[2]:.2f} ms", flush=True)
t0 = time.perf_counter()
for _ in range(5):
    eng.train_step(wav, wl, tg, tl, None)
torch.cuda.synchronize()
print(f"back-to-back {1e3 * (time.perf_counter() - t0) / 5:.2f} ms/step", flush=True)
pr = cProfile.Profile()
pr.enable()
eng.train_step(wav, wl, tg, tl, None)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(top)
st.sort_stats("cumulative").print_stats(top)
