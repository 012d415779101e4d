"""Register-spill / serialized-load scan of every kernel in csrc/ (gfx950 device assembly via hipcc -S).

For each kernel: VGPRs, scratch bytes, and inside its loops (ranges closed by a backward branch) the
scratch reloads and `s_waitcnt vmcnt(0)` drains.  A spilled address reload waits for every load in
flight, so a kernel at the register limit can serialize its staged loads one HBM round trip at a time
(the round-4 dQ kernel: 12 reloads per key block, 65.8 -> 49.1 us once removed).
usage: python tools/isa_scan.py [--all] [name-substring ...]   (default: kernels with scratch or >= 8 drains)
"""
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kd-via-fm-in-asr_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=fast", "-munsafe-fp-atomics",
         f"-I{os.path.join(ROOT, 'include')}", "--offload-device-only", "-S"]


def compile_s(src, out):
    r = subprocess.run([HIPCC, *FLAGS, src, "-o", out], capture_output=True, text=True)
    return out if r.returncode == 0 else None


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.split("\n") if r.returncode == 0 else names


def scan(path):
    lines = open(path).read().split("\n")
    out, i = [], 0
    while i < len(lines):
        m = re.match(r"^(_Z\S+):", lines[i])
        if not m:
            i += 1
            continue
        name, st = m.group(1), i
        e = i
        while e < len(lines) and "s_endpgm" not in lines[e]:
            e += 1
        body = lines[st:e]
        labels = {}
        for k, x in enumerate(body):
            mm = re.match(r"^(\.LBB\w+):", x)
            if mm:
                labels[mm.group(1)] = k
        inloop = [False] * len(body)
        for k, x in enumerate(body):
            mm = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", x)
            if mm:
                t = labels.get(mm.group(1) or mm.group(2), 1 << 30)
                if t < k:
                    for q in range(t, k + 1):
                        inloop[q] = True
        vg = sc = None
        for x in lines[e:e + 2000]:   # the function's register summary follows its code
            if x.startswith("; NumVgprs:") and vg is None:
                vg = int(x.split(":")[1])
            if x.startswith("; ScratchSize:") and sc is None:
                sc = int(x.split(":")[1])
        drains = sum(1 for k, x in enumerate(body) if inloop[k] and "vmcnt(0)" in x)
        reloads = sum(1 for k, x in enumerate(body) if inloop[k] and "scratch_load" in x)
        out.append((name, vg, sc, reloads, drains))
        i = e + 1
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    show_all = "--all" in sys.argv
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with tempfile.TemporaryDirectory() as td, cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda s: compile_s(s, os.path.join(td, os.path.basename(s) + ".s")), srcs))
        rows = []
        for src, o in zip(srcs, outs):
            if o is None:
                print(f"{os.path.basename(src)}: hipcc failed")
                continue
            for r in scan(o):
                rows.append((os.path.basename(src),) + r)
    names = demangle([r[1] for r in rows])
    print(f"{'file':14s} {'vgpr':>4s} {'scratch':>7s} {'loop reloads':>12s} {'loop vmcnt(0)':>13s}  kernel")
    for r, dn in zip(rows, names):
        f, _, vg, sc, rl, dr = r
        dn = dn.replace("kdfm::(anonymous namespace)::", "")
        if args and not any(a in dn for a in args):
            continue
        if not show_all and not args and not (sc or dr >= 8):
            continue
        print(f"{f:14s} {vg if vg is not None else -1:4d} {sc if sc is not None else -1:7d} {rl:12d} {dr:13d}  {dn[:110]}")


if __name__ == "__main__":
    main()
