"""Per-kernel MFMA busy and wave-state shares from the rocprofv3 --pmc passes of tools/pmc_mfma.sh.

  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CU_CYCLES * 4)   fraction of the SIMD-cycles of the
               CUs the kernel kept busy in which an MFMA executed (32 cycles per 32x32x16 bf16,
               MI355X_MICROARCH.md 'SQ PMC units')
  wait / inst_stall / active / lds_stall = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY /
               SQ_WAIT_INST_LDS as shares of SQ_WAVE_CYCLES (the first three are disjoint)
Counters are summed over a kernel's launches (every launch of the 2 profiled steps).
Writes <dir>/mfma.json.  usage: python tools/pmc_mfma.py gpurun_out/<tag>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = (row.get("Kernel_Name") or "").replace("(anonymous namespace)::", "").replace("void ", "")
                cname = row.get("Counter_Name") or ""
                cval = row.get("Counter_Value")
                if not name or not cname or cval is None:
                    continue
                key = name.split("(")[0]
                per[key][cname] += float(cval)
                n[key].add(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(n[key]))
    return per, {k: len(v) for k, v in n.items()}


def main():
    d = sys.argv[1]
    per, n = load(d)
    rows = []
    for k, c in per.items():
        busy = c.get("SQ_BUSY_CU_CYCLES", 0.0)
        wave = c.get("SQ_WAVE_CYCLES", 0.0)
        rows.append({
            "kernel": k, "launches": n.get(k, 0),
            "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (4.0 * busy) if busy else None,
            "wait": c.get("SQ_WAIT_ANY", 0.0) / wave if wave else None,
            "inst_stall": c.get("SQ_WAIT_INST_ANY", 0.0) / wave if wave else None,
            "active": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wave if wave else None,
            "lds_stall": c.get("SQ_WAIT_INST_LDS", 0.0) / wave if wave else None,
            "waves": c.get("SQ_WAVES", 0.0), "busy_cu_cycles": busy, "wave_cycles": wave,
        })
    rows.sort(key=lambda r: -(r["busy_cu_cycles"] or 0.0))
    f = lambda v: "   -  " if v is None else f"{v:6.3f}"  # noqa: E731
    print(f"{'kernel':58s} {'n':>4s} {'mfma':>6s} {'wait':>6s} {'stall':>6s} {'activ':>6s} {'lds':>6s}")
    for r in rows[:40]:
        print(f"{r['kernel'][:58]:58s} {r['launches']:4d} {f(r['mfma_busy'])} {f(r['wait'])} {f(r['inst_stall'])} "
              f"{f(r['active'])} {f(r['lds_stall'])}")
    with open(os.path.join(d, "mfma.json"), "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
