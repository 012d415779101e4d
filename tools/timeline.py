"""Per-stream busy time and critical-path view of one training step from a rocprofv3 kernel trace
(--kernel-trace, rocpd .db or --output-format csv).
usage: python tools/timeline.py <run_results.db | kernel_trace.csv>
Steps are delimited by the CTC kernel (one launch per step); the last full step is analysed."""
import csv
import sqlite3
import sys
from collections import defaultdict


def load(path):
    """(start, end, stream, kernel) rows of a rocpd .db or a kernel_trace.csv, sorted by start."""
    rows = []
    clean = lambda n: n.replace("kdfm::(anonymous namespace)::", "").split("(")[0]  # noqa: E731
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, st, en, sid, qid in c.execute("select name, start, end, stream_id, queue_id from kernels"):
            rows.append((int(st), int(en), str(sid if sid is not None else qid), clean(name)))
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                sid = r.get("Stream_Id") or r.get("Queue_Id") or "0"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), sid, clean(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    rows = load(sys.argv[1])
    # step boundaries: the adamw kernel ends every step
    ends = [e for s, e, q, n in rows if n.startswith("adamw_kernel") or "adamw_kernel" in n]
    if len(ends) < 3:
        print("need >= 3 steps in the trace")
        return
    t0, t1 = ends[-3], ends[-2]
    step = [(s, e, q, n) for s, e, q, n in rows if s >= t0 and e <= t1]
    span = (t1 - t0) / 1e6
    print(f"step window {span:.3f} ms, {len(step)} kernels")
    busy = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, q, n in step:
        busy[q] += (e - s) / 1e6
        cnt[q] += 1
    for q in sorted(busy, key=lambda k: -busy[k]):
        print(f"  stream {q}: busy {busy[q]:8.3f} ms  ({busy[q] / span * 100:5.1f}% of step)  {cnt[q]} kernels")
    # union of busy intervals (any stream running)
    ivs = sorted((s, e) for s, e, q, n in step)
    tot, cs, ce = 0, None, None
    for s, e in ivs:
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            tot += ce - cs
            cs, ce = s, e
    if cs is not None:
        tot += ce - cs
    print(f"  GPU busy (any stream): {tot / 1e6:.3f} ms = {tot / 1e6 / span * 100:.1f}% of the step; idle {span - tot / 1e6:.3f} ms")
    # top kernels per stream
    for q in sorted(busy, key=lambda k: -busy[k]):
        agg = defaultdict(float)
        for s, e, qq, n in step:
            if qq == q:
                agg[n] += (e - s) / 1e6
        top = sorted(agg.items(), key=lambda kv: -kv[1])[:8]
        print(f"  stream {q} top: " + "; ".join(f"{n[:40]} {t:.2f}" for n, t in top))


def producer(step, main, t_prev_end, t_next, slack_us=8.0):
    """The kernel a main-stream gap most likely waited for: the latest-ending kernel on another stream
    that finished inside the gap and at most `slack_us` before the main stream resumed (a cross-stream
    event wait resumes within a few microseconds of its producer's end).  None: nothing on another
    stream ended right before the resume -- the gap is host issue (or a launch the trace cannot see)."""
    best = None
    for s, e, q, n in step:
        if q != main and t_prev_end <= e <= t_next and (t_next - e) / 1e3 <= slack_us:
            if best is None or e > best[0]:
                best = (e, q, n)
    return best


def seq(path):
    """The busiest stream's kernels of the last full step in issue order: gap before each, duration, name; then
    the gap histogram (kernel-boundary idle time by size)."""
    rows = load(path)
    ends = [e for s, e, q, n in rows if "adamw_kernel" in n]
    if len(ends) < 3:
        print("need >= 3 steps in the trace")
        return
    t0, t1 = ends[-3], ends[-2]
    step = [(s, e, q, n) for s, e, q, n in rows if s >= t0 and e <= t1]
    busy = defaultdict(float)
    for s, e, q, n in step:
        busy[q] += e - s
    main_sid = max(busy, key=busy.get)
    prev = t0
    hist = defaultdict(float)
    nh = defaultdict(int)
    for s, e, q, n in step:
        if q != main_sid:
            continue
        g = max(0, s - prev) / 1e3
        b = "<5" if g < 5 else "5-10" if g < 10 else "10-30" if g < 30 else ">=30"
        hist[b] += g
        nh[b] += 1
        print(f"{g:8.1f} {(e - s) / 1e3:8.1f}  {n[:70]}")
        prev = e
    print("gaps before main-stream kernels (us): " + ", ".join(f"{k}: {nh[k]} / {hist[k]:.0f}" for k in
                                                             ("<5", "5-10", "10-30", ">=30")))


def gaps(path, main_sid=None, min_us=30.0):
    """Main-stream idle gaps inside the last full step, each attributed to the producer it waited on
    (producer()): cross-stream waits summed per producer stream / kernel, the rest as host issue."""
    rows = load(path)
    ends = [e for s, e, q, n in rows if "adamw_kernel" in n]
    t0, t1 = ends[-3], ends[-2]
    step = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    busy = defaultdict(float)
    for s, e, q, n in step:
        busy[q] += e - s
    main = main_sid or max(busy, key=busy.get)
    mk = [(s, e, n) for s, e, q, n in step if q == main]
    total = 0.0
    agg = defaultdict(float)
    prev_end, prev_name = t0, "step start"
    out = []
    by_prod = defaultdict(float)
    allgap = 0.0
    for s, e, n in mk:
        g = (s - prev_end) / 1e3
        if g > 0:
            allgap += g
        if g > min_us:
            others = defaultdict(float)
            for s2, e2, q2, n2 in step:
                if q2 != main and e2 > prev_end and s2 < s:
                    others[f"{q2}:{n2[:28]}"] += (min(e2, s) - max(s2, prev_end)) / 1e3
            top = sorted(others.items(), key=lambda kv: -kv[1])[:3]
            pr = producer(step, main, prev_end, s)
            who = f"waits {pr[1]}:{pr[2][:34]}" if pr else "host issue"
            by_prod[who] += g
            out.append((g, prev_name[:30], n[:30], top, who))
            total += g
            for k, v in others.items():
                agg[k.split(":")[0]] += v
        prev_end, prev_name = max(prev_end, e), n
    span = (t1 - t0) / 1e6
    print(f"main stream {main}: idle {allgap / 1e3:.3f} ms of the {span:.3f} ms step; {len(out)} gaps > {min_us} us, "
          f"{total / 1e3:.3f} ms total")
    print("  attributed (gaps > min_us), by producer:")
    for who, g in sorted(by_prod.items(), key=lambda kv: -kv[1])[:20]:
        print(f"    {g / 1e3:7.3f} ms  {who}")
    for g, a, b, top, who in sorted(out, key=lambda x: -x[0])[:25]:
        print(f"  {g:8.1f} us after {a:30s} before {b:30s} [{who}] | " + "; ".join(f"{k} {v:.0f}" for k, v in top))


if __name__ == "__main__":
    main()
    if len(sys.argv) > 2 and sys.argv[2] == "gaps":
        gaps(sys.argv[1])
    elif len(sys.argv) > 2 and sys.argv[2] == "seq":
        seq(sys.argv[1])
