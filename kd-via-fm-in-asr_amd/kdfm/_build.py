"""Build libkdfm.so in-tree with hipcc for gfx950 (no torch extension, no JIT cache).

Each csrc/*.hip is compiled to an object in csrc/build/ in parallel, then linked into
kdfm/libkdfm.so.  Objects are rebuilt when the source or any header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)  # kd-via-fm-in-asr_amd/
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(os.path.dirname(ROOT), "include")
LIB_PATH = os.path.join(PKG_DIR, "libkdfm.so")
IO_LIB_PATH = os.path.join(PKG_DIR, "libkdfm_io.so")
IO_SRC = os.path.join(CSRC, "audio_io.cpp")
CXX = os.environ.get("CXX", "g++")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast",
          "-munsafe-fp-atomics", "-Wno-unused-result", f"-I{INCLUDE}"]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + [h for h in glob.glob(os.path.join(INCLUDE, "*.h"))
                                                   if not h.endswith("kdfm_io.h")]


def _compile(src: str, obj: str) -> str:
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stderr[-6000:]}")
    return obj


def build_io(verbose: bool = False) -> str:
    """libkdfm_io.so: the host-only audio decode / collate library (include/kdfm_io.h), g++."""
    hdr = os.path.join(INCLUDE, "kdfm_io.h")
    src_mtime = max(os.path.getmtime(IO_SRC), os.path.getmtime(hdr))
    if os.path.exists(IO_LIB_PATH) and os.path.getmtime(IO_LIB_PATH) >= src_mtime:
        return IO_LIB_PATH
    cmd = [CXX, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", f"-I{INCLUDE}",
           IO_SRC, "-o", IO_LIB_PATH]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed for audio_io.cpp:\n{r.stderr[-6000:]}")
    if verbose:
        print("linked", IO_LIB_PATH)
    return IO_LIB_PATH


def build(verbose: bool = False, jobs: int | None = None) -> str:
    build_io(verbose)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if not srcs:
        raise RuntimeError(f"no HIP sources under {CSRC}")
    bdir = os.path.join(CSRC, "build")
    os.makedirs(bdir, exist_ok=True)
    hdr_mtime = max((os.path.getmtime(h) for h in _headers()), default=0.0)
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(bdir, os.path.basename(s).replace(".hip", ".o"))
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_mtime):
            todo.append((s, o))
    jobs = jobs or min(8, max(1, len(todo)))
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            futs = [ex.submit(_compile, s, o) for s, o in todo]
            for f in futs:
                o = f.result()
                if verbose:
                    print("compiled", os.path.basename(o))
    lib_mtime = os.path.getmtime(LIB_PATH) if os.path.exists(LIB_PATH) else -1.0
    if todo or lib_mtime < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB_PATH, *objs, "-L/opt/rocm/lib",
               "-Wl,-rpath,/opt/rocm/lib", "-lrocprofiler-sdk-roctx"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        if verbose:
            print("linked", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose=True))
