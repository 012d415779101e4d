"""Kernel-time census of one eager ver5 step, attributed to the calling source line.

Every libkdfm entry point is bracketed with HIP events on the launch stream (the teacher runs on
the main stream here so that everything is serialised); GEMMs are labelled with M, N, K, batch and
split-K.  usage: python tools/census.py [top]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 60
cfg = DEFAULT
K.set_math(cfg.math)
eng = Ver5Engine(cfg, "cuda")
B, N, U = 32, 256000, 100
wav, wl, tg, tl = synthetic_batch(cfg, B, N, U, "cuda")
eng.train_step(wav, wl, tg, tl)
torch.cuda.synchronize()

records = []
_orig_call = _lib.call
_orig_gemm_call = None


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        f = os.path.basename(fr.filename)
        if f in ("kernels.py", "_lib.py", "census.py"):
            continue
        return f"{f}:{fr.lineno}:{fr.name}"
    return "?"


def timed_call(name, *args):
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    label = name
    if name == "kdfm_gemm":
        d = args[0]._obj if hasattr(args[0], "_obj") else None
        if d is not None:
            label = (f"gemm M={d.M} N={d.N} K={d.K} b={d.batch1 * d.batch2} sk={d.splitk} "
                     f"a={d.amode} b={d.bmode}")
    s.record()
    _orig_call(name, *args)
    e.record()
    records.append((site(), label, s, e))


_lib.call = timed_call
K.call = timed_call
for _ in range(2):
    records.clear()
    eng.train_step(wav, wl, tg, tl)
    torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for st, label, s, e in records:
    ms = s.elapsed_time(e)
    tot += ms
    a = agg[(st, label)]
    a[0] += 1
    a[1] += ms
print(f"total {tot:.3f} ms over {len(records)} calls")
for (st, label), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{ms:8.3f} ms  {n:4d}x  {ms / n * 1e3:8.1f} us  {st:45s} {label}")
by_file = collections.defaultdict(float)
for (st, label), (n, ms) in agg.items():
    by_file[st.split(":")[0] + ":" + st.split(":")[2]] += ms
print("\nby function:")
for k, v in sorted(by_file.items(), key=lambda kv: -kv[1])[:30]:
    print(f"{v:8.3f} ms  {k}")
