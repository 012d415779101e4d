"""Per-kernel HBM traffic from the two rocprofv3 --pmc passes written by tools/pmc_traffic.sh.

bytes/launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   (FETCH_SIZE / WRITE_SIZE are in KiB; on
gfx950 FETCH_SIZE counts half the bytes of a 16-B/lane streaming read, MI355X_MICROARCH.md §HBM, so
the read side is doubled).  Kernels are keyed by name (+ grid for the generic GEMM, like
prof_summary.py).  Also writes <dir>/traffic.json for bench.py / DESIGN.md.
usage: python tools/pmc_summary.py gpurun_out/<tag>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pattern):
    files = glob.glob(pattern, recursive=True)
    if not files:
        raise SystemExit(f"no counter csv matches {pattern}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("kernel_name") or ""
                cval = row.get("Counter_Value") or row.get("counter_value")
                if not name or cval is None:
                    continue
                name = name.replace("(anonymous namespace)::", "").replace("void ", "")
                key = name.split("(")[0]
                gx = row.get("Grid_Size_X") or row.get("Grid_Size") or ""
                wg = row.get("Workgroup_Size_X") or row.get("Workgroup_Size") or ""
                if "gemm_kernel" in name and gx and wg:
                    key = f"{key} grid={int(gx) // max(1, int(wg))}x{row.get('Grid_Size_Y', '1')}"
                per[key].append(float(cval))
    return per


def main():
    d = sys.argv[1]
    fetch = load(os.path.join(d, "fetch", "**", "*counter_collection.csv"))
    write = load(os.path.join(d, "write", "**", "*counter_collection.csv"))
    rows = []
    for k in set(fetch) | set(write):
        f = fetch.get(k, [])
        w = write.get(k, [])
        n = max(len(f), len(w))
        fb = 2.0 * 1024.0 * (sum(f) / len(f)) if f else 0.0
        wb = 1024.0 * (sum(w) / len(w)) if w else 0.0
        rows.append({"kernel": k, "launches": n, "read_bytes": fb, "write_bytes": wb,
                     "bytes_per_launch": fb + wb, "bytes_total": (fb + wb) * n})
    rows.sort(key=lambda r: -r["bytes_total"])
    print(f"{'kernel':60s} {'launches':>8s} {'MB read/l':>10s} {'MB write/l':>10s} {'MB total':>10s}")
    for r in rows:
        print(f"{r['kernel'][:60]:60s} {r['launches']:8d} {r['read_bytes'] / 1e6:10.2f} "
              f"{r['write_bytes'] / 1e6:10.2f} {r['bytes_total'] / 1e6:10.1f}")
    with open(os.path.join(d, "traffic.json"), "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
