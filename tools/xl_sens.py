"""bench.py's two FastConformer-XL sensitivity lines (bf16, then MX fp8 products) back to back in one process, in
both orders: whether the order or the process's earlier work moves either number."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    for fp8 in (False, True, False, True):
        r = bench.sensitivity(dev, bench.N_SAMPLES, linear_fp8=fp8,
                              **bench.XL_SHAPES)
        print(f"fp8={fp8}: {r['value']} utt/s, {r['ms_per_step']} ms/step", flush=True)


if __name__ == "__main__":
    main()
