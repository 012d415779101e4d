"""Where does the host block while replaying the bench's step plan?  Times every op of
StepPlan.replay (kernel launch, event record / wait, host callback) back to back over several steps
and prints (a) the host time at which each op was issued, relative to the step start, for the
slowest-to-issue ops and (b) the cumulative issue time.  A launch that takes hundreds of
microseconds to return means the host blocked in the runtime (a full hardware queue, a blocking
event call), so every later launch -- whatever its stream -- issues late.
usage: python tools/plan_issue_probe.py [steps] [top]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402
from kdfm.engine import Ver5Engine, synthetic_batch  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda", 0)
K.set_math(DEFAULT.math)
eng = Ver5Engine(DEFAULT, dev)
wav, wl, tg, tl = synthetic_batch(DEFAULT, 32, 256000, 100, dev, seed=1234)
eng.train_step(wav, wl, tg, tl, None)
plan = eng.make_plan(wav, wl, tg, tl)
torch.cuda.synchronize()
names = {}
streams = {eng.compute_stream.cuda_stream: "compute", eng._side_stream().cuda_stream: "teacher"}
from kdfm.overlap import WGRAD  # noqa: E402
for st in WGRAD._side.values():
    streams[st.cuda_stream] = "wgrad"


def label(op):
    if op[0] == "k":
        nm = getattr(op[1], "__name__", "?")
        s = op[2][-1] if op[2] else None
        s = s.value if hasattr(s, "value") else s
        return f"{nm} [{streams.get(s, s)}]"
    if op[0] in ("er", "ew"):
        s = op[2].value
        return f"{'record' if op[0] == 'er' else 'wait'} [{streams.get(s, s)}]"
    return f"host {getattr(op[1], '__name__', op[1])}"


rec, wt = plan._ev_record, plan._ev_wait
worst = {}
totals = []
for it in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    times = []
    for i, op in enumerate(plan.ops):
        a = time.perf_counter()
        if op[0] == "k":
            if op[3] != K.get_deterministic():
                K.set_deterministic(op[3])
            op[1](*op[2])
        elif op[0] == "er":
            rec(op[1], op[2])
        elif op[0] == "ew":
            wt(op[2], op[1])
        else:
            op[1](*op[2])
        b = time.perf_counter()
        times.append((b - a, a - t0, i))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    totals.append((t1 - t0, t2 - t0))
    if it >= 2:
        for dt, at, i in times:
            if dt > worst.get(i, (0, 0))[0]:
                worst[i] = (dt, at)
print(f"{len(plan.ops)} ops; per step: issue {1e3 * min(t[0] for t in totals[2:]):.2f} ms, "
      f"issue + drain {1e3 * min(t[1] for t in totals[2:]):.2f} ms")
print("slowest ops to issue (max over steps >= 2): us, issued at ms into the step, op index, op")
for i, (dt, at) in sorted(worst.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"  {1e6 * dt:9.1f} us  at {1e3 * at:7.3f} ms  #{i:5d}  {label(plan.ops[i])}")
# cumulative issue curve: when was each 10% of the ops issued
n = len(plan.ops)
print("issue progress (last step): " + ", ".join(f"{int(100 * k / 10)}% at {1e3 * times[min(n - 1, k * n // 10)][1]:.2f} ms"
                                                  for k in range(1, 11)))
