"""Recompute the bench line's per-family roofline figures from a rocprofv3 kernel trace of the same command
(the line's timings must follow from profiles/).

usage: python tools/roofline_check.py <bench log or JSON line file> <kernel_trace.csv | results.db>

For every family of `roofline_by_family` (and the headline `roofline` family): the kernel time per step of the
family's kernels in the trace (whole steps only, tools/prof_summary.py's window; the folds and row-dot prologues
count toward their family), against the line's own ms/step, which the bench takes from HIP events around every
launch of a replayed step plan; the achieved rate the line reports, and the rate its algorithmic bytes / FLOPs give
over the trace's time.  |ratio - 1| <= 0.10 is the agreement asked for."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from prof_summary import rows  # noqa: E402


def families():
    import bench
    fam = dict(bench.ROUTE_KERNELS)
    fam.update(bench.FAMILY_KERNELS)
    fam["wgrad_rows"] = tuple(set(bench.ROUTE_KERNELS["wgrad_rows"]) | set(bench.FAMILY_KERNELS["wgrad_bf16"]))
    fam["big"] = ("big_gemm_kernel", "big_fold_kernel")
    return fam


def base(name):
    n = name.replace("kdfm::(anonymous namespace)::", "").replace("kdfm::", "")
    n = n.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0].strip()


def main():
    line = None
    with open(sys.argv[1]) as fh:
        for ln in fh:
            ln = ln.strip()
            if ln.startswith("{") and '"roofline"' in ln:
                line = json.loads(ln)
    assert line is not None, "no bench JSON line"
    allr = sorted(rows(sys.argv[2]), key=lambda r: r[5])
    ends = [r[6] for r in allr if "adamw_kernel" in r[0]]
    lo, hi = ends[0], ends[-1]
    steps = len(ends) - 1
    win = [r for r in allr if r[5] >= lo and r[6] <= hi]
    fam = families()
    per = {}
    for name, d, *_ in win:
        b = base(name)
        for f, stems in fam.items():
            if b in stems:
                per.setdefault(f, [0.0, 0])
                per[f][0] += d
                per[f][1] += 1
    print(f"trace: {steps} whole steps, {len(win) / steps:.0f} launches/step")
    print(f"{'family':12s} {'line ms/step':>12s} {'trace ms/step':>13s} {'ratio':>6s}  line rate -> rate over the trace's time")
    worst = 0.0
    for f, v in line["roofline_by_family"].items():
        t = per.get(f)
        if not t:
            print(f"{f:12s} {v['ms_per_step']:12.3f} {'-':>13s}")
            continue
        tms = t[0] / steps / 1e6
        ratio = v["ms_per_step"] / tms if tms > 0 else float("nan")
        tot_b = v["bytes_per_launch"] * v["launches"]
        tot_f = v["flops_per_launch"] * v["launches"]
        gbps = tot_b / (tms * 1e-3) / 1e9
        tfl = tot_f / (tms * 1e-3) / 1e12
        print(f"{f:12s} {v['ms_per_step']:12.3f} {tms:13.3f} {ratio:6.3f}  {v['GB_per_s']:8.1f} -> {gbps:8.1f} GB/s, "
              f"{v['TFLOP_per_s']:7.2f} -> {tfl:7.2f} TFLOP/s")
        if v["ms_per_step"] > 0.3:
            worst = max(worst, abs(ratio - 1.0))
    r = line["roofline"]
    dom = r["kernel"].split(" family")[0]
    t = per.get(dom)
    if t:
        tms = t[0] / steps / 1e6
        v = line["roofline_by_family"][dom]
        ach = (v["bytes_per_launch"] * v["launches"] / (tms * 1e-3) / 1e9) if r["unit"] == "GB/s" else \
            (v["flops_per_launch"] * v["launches"] / (tms * 1e-3) / 1e12)
        print(f"headline roofline family {dom}: line achieved {r['achieved']} {r['unit']} (frac {r['frac']}) -> over the "
              f"trace's time {ach:.1f} {r['unit']} (frac {ach / r['peak']:.4f}); ratio {r['achieved'] / ach:.3f}")
    print(f"worst |ratio - 1| over families with >= 0.3 ms/step: {worst:.3f}")


if __name__ == "__main__":
    main()
