"""Summarise a rocprofv3 kernel trace (rocpd .db or --output-format csv kernel_trace.csv): kernel
time per step grouped by kernel (+GEMM template and grid).
usage: python tools/prof_summary.py <run_results.db | run_kernel_trace.csv> [steps] [top]
Only whole steps are summarised: the launches between the end of the first fused AdamW launch and the
end of the last one, divided by the number of optimizer steps in between (a fixed "5" over a
9-step trace overstated every per-step figure 1.8x, and the engine-construction copies before the first
step -- the "94 copyBuffer launches per step" -- were never step work); an explicit `steps` that disagrees
is reported and ignored."""
import collections
import csv
import sqlite3
import sys


def rows(path):
    """(name, duration, grid x in workgroups, grid y, grid z, start, end) of every dispatch."""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, st, en, gx, gy, gz, wx in c.execute(
                "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels"):
            yield name, int(en) - int(st), int(gx) // max(int(wx), 1), int(gy), int(gz), int(st), int(en)
    else:
        for r in csv.DictReader(open(path)):
            wx = int(r.get("Workgroup_Size_X", 256) or 256)
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            yield (r["Kernel_Name"], en - st, int(r["Grid_Size_X"]) // wx, int(r["Grid_Size_Y"]),
                   int(r["Grid_Size_Z"]), st, en)


def main():
    path = sys.argv[1]
    nsteps = float(sys.argv[2]) if len(sys.argv) > 2 and float(sys.argv[2]) > 0 else None
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
    allr = sorted(rows(path), key=lambda r: r[5])
    # whole steps only: from the end of the first optimizer step to the end of the last one (setup work
    # before the first step -- engine construction, parameter loads, plan recording's allocations -- and
    # the bench's post-step sensitivity runs are outside every step)
    ends = [r[6] for r in allr if "adamw_kernel" in r[0]]
    if len(ends) >= 2:
        lo, hi = ends[0], ends[-1]
        outside = [r for r in allr if not (r[5] >= lo and r[6] <= hi)]
        allr = [r for r in allr if r[5] >= lo and r[6] <= hi]
        nopt = len(ends) - 1
        print(f"window: {nopt} whole steps (first optimizer step end .. last); {len(outside)} launches outside "
              f"({sum(r[1] for r in outside) / 1e6:.3f} ms) excluded")
    else:
        nopt = len(ends)
    agg = collections.defaultdict(lambda: [0, 0.0])
    tot, nl = 0.0, 0
    for name, d, gx, gy, gz, st, en in allr:
        n = name.replace("kdfm::(anonymous namespace)::", "").replace("kdfm::", "")
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
    print(f"  gemm share: {gemm / max(tot, 1) * 100:.1f}%")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / nsteps / 1e6:8.3f} ms/step  {v[0] / nsteps:6.1f}/step  avg {v[1] / v[0] / 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
