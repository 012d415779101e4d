"""Summarise a rocprofv3 kernel trace (rocpd .db or --output-format csv kernel_trace.csv): kernel
time per step grouped by kernel (+GEMM template and grid).
usage: python tools/prof_summary.py <run_results.db | run_kernel_trace.csv> [steps] [top]
The step count is the number of fused AdamW launches the trace holds (one per optimizer step: the
bench's eager warm-up, the recorded plan step, the warm-up and timed replays and the instrumented
step all count); an explicit `steps` that disagrees with it is reported and ignored (a
fixed "5" over a 9-step trace overstated every per-step figure 1.8x)."""
import collections
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, gx, gy, gz, wx in c.execute(
                "select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels"):
            yield name, int(dur), int(gx) // max(int(wx), 1), int(gy), int(gz)
    else:
        for r in csv.DictReader(open(path)):
            wx = int(r.get("Workgroup_Size_X", 256) or 256)
            yield (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                   int(r["Grid_Size_X"]) // wx, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))


def main():
    path = sys.argv[1]
    nsteps = float(sys.argv[2]) if len(sys.argv) > 2 and float(sys.argv[2]) > 0 else None
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
    agg = collections.defaultdict(lambda: [0, 0.0])
    tot, nl, nopt = 0.0, 0, 0
    for name, d, gx, gy, gz in rows(path):
        n = name.replace("kdfm::(anonymous namespace)::", "").replace("kdfm::", "")
        if "adamw_kernel" in n:
            nopt += 1
        tot += d
        nl += 1
        base = n.split("(")[0]
        key = base + (f" grid=({gx},{gy},{gz})" if "gemm" in n else "")
        agg[key][0] += 1
        agg[key][1] += d
    if nopt and nsteps and nsteps != nopt:
        print(f"note: {nsteps:g} steps given but the trace holds {nopt} optimizer steps; using {nopt}")
    nsteps = nopt or nsteps or 1
    print(f"steps={nsteps:g}  total kernel time per step: {tot / nsteps / 1e6:.3f} ms  ({nl / nsteps:.0f} launches/step)")
    gemm = sum(v[1] for k, v in agg.items() if "gemm" in k)
    print(f"  gemm share: {gemm / tot * 100:.1f}%")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / nsteps / 1e6:8.3f} ms/step  {v[0] / nsteps:6.1f}/step  avg {v[1] / v[0] / 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
