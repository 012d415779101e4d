"""How much of the step does the frozen teacher's encoder cost on the critical path?  Times the bench
step (eager and step-plan replay) as is and with the teacher encoder's launches skipped (its features
stay whatever the previous step left: timing only, the numbers are not a training step).  The gap is
the most a schedule that computes the teacher one step ahead (overlapping the previous step's
backward) could gain.
usage: python tools/teacher_ahead_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import engine as E  # noqa: E402
from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
K.set_math(DEFAULT.math)
orig = E.encoder_forward_steps
skip = {"on": False}


def patched(cfg, S, P, prefix, *a, **k):
    if skip["on"] and prefix.startswith("teacher."):
        def idle():
            for _ in range(cfg.n_layers + 1):
                yield
        return idle()
    return orig(cfg, S, P, prefix, *a, **k)


E.encoder_forward_steps = patched


def run(label):
    eng = E.Ver5Engine(DEFAULT, dev)
    wav, wl, tg, tl = E.synthetic_batch(DEFAULT, 32, 256000, 100, dev, seed=1234)
    for _ in range(3):
        eng.train_step(wav, wl, tg, tl)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.train_step(wav, wl, tg, tl)
    torch.cuda.synchronize()
    eager = 1e3 * (time.perf_counter() - t0) / steps
    plan = eng.make_plan(wav, wl, tg, tl)
    for _ in range(2):
        plan.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.replay()
    torch.cuda.synchronize()
    rep = 1e3 * (time.perf_counter() - t0) / steps
    print(f"{label}: eager {eager:.2f} ms/step, plan replay {rep:.2f} ms/step", flush=True)
    del plan, eng
    torch.cuda.empty_cache()


run("with the teacher encoder")
skip["on"] = True
run("teacher encoder skipped")
