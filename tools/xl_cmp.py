"""Why bench.py's xl_fp8_sensitivity reads slower than tools/xl_step.py: the same MX-fp8 XL engine timed (a) by
bench.sensitivity, (b) per step with a sync after each (xl_step.py's way), (c) 3 steps back to back."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from dataclasses import replace

    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.engine import Ver5Engine, synthetic_batch
    dev = torch.device("cuda")
    fp8 = len(sys.argv) < 2 or sys.argv[1] == "fp8"
    r = bench.sensitivity(dev, bench.N_SAMPLES, linear_fp8=fp8, **bench.XL_SHAPES)
    print(f"(a) bench.sensitivity fp8={fp8}: {r['ms_per_step']} ms/step", flush=True)
    if len(sys.argv) > 2 and sys.argv[2] == "clear":   # drop every module-level device cache before the second engine
        n = (len(K._BF16_W), len(K._FP8_W), len(K._SCRATCH), len(K._RETIRED))
        K._BF16_W.clear(); K._FP8_W.clear(); K._SCRATCH.clear(); K._RETIRED.clear()  # noqa: E702
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        print(f"cleared caches (bf16 copies, fp8 copies, scratch, retired) = {n}; "
              f"allocated {torch.cuda.memory_allocated() / 2**30:.1f} GiB", flush=True)
    else:
        print(f"allocated {torch.cuda.memory_allocated() / 2**30:.1f} GiB, reserved "
              f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB", flush=True)
    cfg = replace(DEFAULT, linear_fp8=fp8, **bench.XL_SHAPES)
    eng = Ver5Engine(cfg, dev)
    eng.set_seed(1000)
    wav, wl, tg, tl = synthetic_batch(cfg, 32, bench.N_SAMPLES, 100, dev, seed=1234)
    with K.mode(cfg.math, fp8=cfg.linear_fp8):
        eng.train_step(wav, wl, tg, tl)
        torch.cuda.synchronize()
        for i in range(3):
            t0 = time.perf_counter()
            eng.train_step(wav, wl, tg, tl)
            torch.cuda.synchronize()
            print(f"(b) step {i}: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
        t0 = time.perf_counter()
        for i in range(3):
            eng.train_step(wav, wl, tg, tl)
        torch.cuda.synchronize()
        print(f"(c) 3 back-to-back: {1e3 * (time.perf_counter() - t0) / 3:.1f} ms/step", flush=True)


if __name__ == "__main__":
    main()
