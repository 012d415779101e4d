"""Summarise a rocprofv3 --kernel-trace CSV: kernel time per step grouped by kernel (+GEMM template
and grid).  usage: python tools/prof_summary.py <run_kernel_trace.csv> <steps_in_trace> [top]"""
import collections
import csv
import sys

path, nsteps = sys.argv[1], float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for r in rows:
    n = r["Kernel_Name"].replace("kdfm::(anonymous namespace)::", "")
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot += d
    if "gemm" in n:
        key = n.split("(")[0] + f" grid=({int(r['Grid_Size_X']) // 256},{r['Grid_Size_Y']},{r['Grid_Size_Z']})"
    else:
        key = n.split("(")[0]
    agg[key][0] += 1
    agg[key][1] += d
print(f"total kernel time per step: {tot / nsteps / 1e6:.3f} ms  ({len(rows) / nsteps:.0f} launches/step)")
gemm = sum(v[1] for k, v in agg.items() if "gemm" in k)
print(f"  gemm share: {gemm / tot * 100:.1f}%")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{v[1] / nsteps / 1e6:8.3f} ms/step  {v[0] / nsteps:6.1f}/step  avg {v[1] / v[0] / 1e3:8.1f} us  {k}")
