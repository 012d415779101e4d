"""The FastConformer-XL shape step (bench.py XL_SHAPES: d_model 1024, 8 heads, 24 layers, dw_striding x8, B=32 x 16 s)
run eagerly for a few steps: per-step time (HIP events) and, under rocprofv3 --kernel-trace --stats, its kernel
mix.  usage: python tools/xl_step.py [steps] [math]   (math: bf16 | fp8)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, ROOT)
import kdfm  # noqa: E402,F401
import torch  # noqa: E402


def main():
    from dataclasses import replace

    from bench import XL_SHAPES
    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.engine import Ver5Engine, synthetic_batch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    math = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    cfg = replace(DEFAULT, math="bf16", linear_fp8=(math == "fp8"), **XL_SHAPES)
    dev = torch.device("cuda")
    eng = Ver5Engine(cfg, dev)
    eng.set_seed(1000)
    wav, wl, tg, tl = synthetic_batch(cfg, 32, 256000, 100, dev, seed=1234)
    with K.mode(cfg.math, fp8=cfg.linear_fp8):
        eng.train_step(wav, wl, tg, tl)
        torch.cuda.synchronize()
        for i in range(steps):
            t0 = time.perf_counter()
            eng.train_step(wav, wl, tg, tl)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"step {i}: {dt * 1e3:.1f} ms  {32 / dt:.1f} utt/s  losses {eng.losses.tolist()}", flush=True)


if __name__ == "__main__":
    main()
