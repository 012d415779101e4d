"""Runs tests/test_ddp_equiv_gpu.py's bitwise DDP-equivalence check N times in one process (each run spawns its
two gloo ranks) and prints the per-rank result dicts, to catch its intermittent failure with the diagnostics
(worst parameter, shard values).  usage: python tools/ddp_equiv_repeat.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "kd-via-fm-in-asr_amd")]

import torch.multiprocessing as mp  # noqa: E402

import test_ddp_equiv_gpu as T  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    bad = 0
    for i in range(n):
        mgr = mp.Manager()
        out = mgr.dict()
        mp.spawn(T._worker, args=(2, T._free_port(), out), nprocs=2, join=True)
        for r in range(2):
            o = dict(out[r])
            ok = o["grad_equal"] and o["ranks_equal"] and o["ref_equal"]
            bad += 0 if ok else 1
            print(f"run {i} rank {r}: {'ok' if ok else 'MISMATCH'} {o}", flush=True)
        mgr.shutdown()
    print(f"{bad} mismatching rank results over {n} runs", flush=True)


if __name__ == "__main__":
    main()
