"""Happens-before race checker for the multi-stream step (host-side trace, no GPU instrumentation).

Every device memory access the step issues is recorded with the HIP stream it is issued on:

  * libkdfm launches (kernels.call): the read / write sets come from include/kdfm.h itself -- a
    `const T*` parameter is read, a non-const pointer is written -- with each pointer's extent taken
    from the tensor kernels.ptr() resolved it from; kdfm_gemm's descriptor is decoded field by field
    (C, Cpre, loss_acc, ones_out, ws written; A, B, bias, R, aux, seed, mask read);
  * torch ops (a TorchDispatchMode): inputs read, mutated arguments and fresh outputs written, views
    skipped; every fresh output is an ALLOCATION (generation) of its storage range;
  * cross-stream ordering: torch.cuda.Event record / wait (Stream.wait_stream and the engine's
    StreamLinks go through them), torch.cuda.synchronize, Stream / Event synchronize, .item();
  * collectives: torch.distributed.all_reduce is replaced by a model of gloo / RCCL's stream
    semantics (the collective starts after the issuing stream's prior work on a stream of its own and
    work.wait() makes the waiting stream wait for it) so a world of 2 is traced on one process.

Ordering is tracked with vector clocks (one per stream; an event carries the clock of its stream at
record time; a wait merges it).  Two accesses to overlapping bytes conflict when they are on
different streams, at least one writes, and neither happens before the other.  An access to memory
the caching allocator has meanwhile handed to a new tensor (a different generation) is a conflict
only if the old owner's stream never recorded itself on it (Tensor.record_stream makes the allocator
wait for that stream in real time before reuse, which no stream edge shows).

Usage (on the GPU box):  python tools/race_check.py [--layers N] [--batch B] [--seconds S] [--steps K] [--diffkd]
    [--deterministic | --serial] [--plan] [--mutate heads_join|bucket_early|allreduce_caller]
prints one line per distinct conflicting pair (issue site of both accesses) and exits 1 if any.
tests/test_race_gpu.py runs it on the default overlapped schedule (KD heads in two layer halves, the
bucketed all-reduce of a world of 2) with use_diffkd off and on, on the serialised schedule (deterministic
and overlap_wgrad=False, heads split on), on a step plan's recording step, and with each --mutate defect
(which it must report; allreduce_caller is a negative control that must stay clean).
"""
from __future__ import annotations

import argparse
import bisect
import ctypes as C
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
from torch.utils._pytree import tree_flatten  # noqa: E402

PAGE = 1 << 20


# ------------------------------------------------------------------------------------------------
# include/kdfm.h: pointer parameters and their const-ness
# ------------------------------------------------------------------------------------------------

def parse_header(path=os.path.join(ROOT, "include", "kdfm.h")):
    """name -> [(param name, kind)] with kind in {"r", "w", "rr" (host array of read pointers),
    "ww" (host array of written pointers), None (not a device pointer)}."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    out = {}
    for m in re.finditer(r"\b(?:int|int32_t|int64_t|void|const char\*)\s+(kdfm_\w+)\s*\(([^;{]*?)\)\s*;", src, re.S):
        name, params = m.group(1), m.group(2)
        plist = []
        for p in params.split(","):
            p = " ".join(p.split())
            if not p or p == "void":
                continue
            pname = re.findall(r"(\w+)$", p)[0]
            t = p[: -len(pname)].strip()
            if pname == "stream" or t.startswith("char") or "char*" in t.replace(" ", ""):
                kind = None
            elif t.count("*") == 2:
                kind = "rr" if t.startswith("const") else "ww"
            elif "*" in t:
                kind = "r" if t.startswith("const") else "w"
            else:
                kind = None
            plist.append((pname, kind))
        out[name] = plist
    return out


# ------------------------------------------------------------------------------------------------
# vector clocks
# ------------------------------------------------------------------------------------------------

class Access:
    __slots__ = ("lo", "hi", "stream", "clock", "write", "gen", "site", "what")

    def __init__(self, lo, hi, stream, clock, write, gen, site, what):
        self.lo, self.hi, self.stream, self.clock, self.write = lo, hi, stream, clock, write
        self.gen, self.site, self.what = gen, site, what


class Tracer:
    def __init__(self, roles=None):
        self.vc = {}          # stream -> {stream: clock}
        self.floor = {}       # clocks every stream has reached (host synchronisation)
        self.ev = {}          # id(event) -> vc at record
        self.pages = {}       # page -> [Access]
        self.allocs = []      # sorted [(lo, hi, gen, alloc stream, recorded streams)]
        self.alloc_lo = []
        self.ngen = 0
        self.conflicts = {}   # (site a, site b) -> (count, example)
        self.roles = roles if roles is not None else {}
        self.header = parse_header()
        self.recent = {}      # kernels.ptr() spans since the last call
        self.pseudo = 0
        self.active = False
        self.naccess = 0

    # ---- clocks ----
    def _clock(self, s):
        v = self.vc.get(s)
        if v is None:
            v = self.vc[s] = dict(self.floor)
        return v

    def tick(self, s):
        v = self._clock(s)
        v[s] = v.get(s, 0) + 1
        return v[s]

    def record(self, ev, s):
        self.ev[id(ev)] = dict(self._clock(s))

    def wait(self, ev, s):
        e = self.ev.get(id(ev))
        if e is None:
            return
        v = self._clock(s)
        for k, c in e.items():
            if v.get(k, 0) < c:
                v[k] = c

    def sync_all(self):
        for v in self.vc.values():
            for k, c in v.items():
                if self.floor.get(k, 0) < c:
                    self.floor[k] = c
        for v in self.vc.values():
            for k, c in self.floor.items():
                if v.get(k, 0) < c:
                    v[k] = c

    def sync_clock(self, e):
        for k, c in e.items():
            if self.floor.get(k, 0) < c:
                self.floor[k] = c
        for v in self.vc.values():
            for k, c in self.floor.items():
                if v.get(k, 0) < c:
                    v[k] = c

    def hb(self, a: Access, s, v):
        return a.stream == s or v.get(a.stream, 0) >= a.clock

    # ---- allocations ----
    def alloc(self, lo, hi, s):
        i = bisect.bisect_left(self.alloc_lo, lo)
        j = i
        while j > 0 and self.allocs[j - 1][1] > lo:
            j -= 1
        k = i
        while k < len(self.allocs) and self.allocs[k][0] < hi:
            k += 1
        del self.allocs[j:k]
        del self.alloc_lo[j:k]
        self.ngen += 1
        bisect.insort(self.alloc_lo, lo)
        i = self.alloc_lo.index(lo)
        self.allocs.insert(i, (lo, hi, self.ngen, s, set()))
        return self.ngen

    def gen_of(self, p):
        i = bisect.bisect_right(self.alloc_lo, p) - 1
        if i >= 0 and self.allocs[i][0] <= p < self.allocs[i][1]:
            return self.allocs[i]
        return None

    def recorded(self, gen, s):
        for a in self.allocs:
            if a[2] == gen:
                return s in a[4]
        return self._dead_recorded.get((gen, s), False)

    _dead_recorded: dict = {}

    def record_stream(self, p, s):
        a = self.gen_of(p)
        if a is not None:
            a[4].add(s)
            self._dead_recorded[(a[2], s)] = True

    # ---- accesses ----
    def access(self, lo, hi, s, write, site, what):
        if hi <= lo:
            return
        self.naccess += 1
        a = self.gen_of(lo)
        gen = a[2] if a is not None else 0
        v = self._clock(s)
        clock = self.tick(s)
        cur = Access(lo, hi, s, clock, write, gen, site, what)
        seen = set()
        for pg in range(lo // PAGE, (hi - 1) // PAGE + 1):
            lst = self.pages.get(pg)
            if lst is None:
                self.pages[pg] = [cur]
                continue
            keep = []
            for p in lst:
                if id(p) in seen:
                    keep.append(p)
                    continue
                if p.lo < hi and lo < p.hi and (p.write or write) and not self.hb(p, s, v):
                    seen.add(id(p))
                    if p.gen == gen or not self._dead_recorded.get((p.gen, p.stream), False):
                        self._report(p, cur)
                # prune: a covered access that happens before this one (or is on its stream) is
                # subsumed by it for every later check
                covered = lo <= p.lo and p.hi <= hi and (write or (not p.write and p.stream == s))
                if covered and self.hb(p, s, v) and (p.gen == gen):
                    continue
                keep.append(p)
            keep.append(cur)
            self.pages[pg] = keep

    def _role(self, s):
        return self.roles.get(s, f"stream@{s:#x}" if isinstance(s, int) and s >= 0 else str(s))

    def _report(self, p, c):
        key = (p.site, p.what, c.site, c.what)
        n, ex = self.conflicts.get(key, (0, None))
        if ex is None:
            ex = (self._role(p.stream), "W" if p.write else "R", self._role(c.stream), "W" if c.write else "R",
                  max(p.lo, c.lo), min(p.hi, c.hi), p.gen != c.gen)
        self.conflicts[key] = (n + 1, ex)

    def report(self, out=sys.stdout):
        for (ps, pw, cs, cw), (n, ex) in sorted(self.conflicts.items(), key=lambda kv: -kv[1][0]):
            rp, ap, rc, ac, lo, hi, reuse = ex
            print(f"RACE x{n}{' (memory reused)' if reuse else ''}: {ap} {pw} [{rp}] at {ps}\n"
                  f"        vs {ac} {cw} [{rc}] at {cs}   bytes {lo:#x}+{hi - lo}", file=out)
        return len(self.conflicts)


# ------------------------------------------------------------------------------------------------
# hooks
# ------------------------------------------------------------------------------------------------

T: Tracer | None = None
_HERE = os.path.abspath(__file__)


_SKIP = ("kernels.py", "_lib.py", "overlap.py", "race_check.py")


def _site():
    """innermost frame of the product package outside the kernel wrappers (the issue site)."""
    f = sys._getframe(1)
    while f is not None:
        fn = f.f_code.co_filename
        if not fn.endswith(_SKIP) and ("torch" + os.sep) not in fn:
            return f"{os.path.basename(fn)}:{f.f_lineno}"
        f = f.f_back
    return "?"


def _span(t):
    if t.numel() == 0:
        return None
    n = sum((s - 1) * st for s, st in zip(t.shape, t.stride()) if s > 0) + 1
    p = t.data_ptr()
    return p, p + n * t.element_size()


def _cur():
    from kdfm import kernels as K
    return K.stream_ptr()


def _stream_ptr(s):
    if s is None:
        return _cur()
    if hasattr(s, "cuda_stream"):
        return s.cuda_stream
    return torch.cuda.Stream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type).cuda_stream


def install(tracer: Tracer):
    global T
    T = tracer
    from kdfm import kernels as K
    orig_ptr, orig_call = K.ptr, K.call

    def ptr(t):
        p = orig_ptr(t)
        if T.active and p is not None:
            sp = _span(t)
            if sp is not None:
                T.recent[p] = max(T.recent.get(p, sp[1]), sp[1])
        return p

    def call(name, *args):
        if T.active:
            _on_call(name, args)
        T.recent = {}
        return orig_call(name, *args)

    K.ptr, K.call = ptr, call

    E, S = torch.cuda.Event, torch.cuda.Stream
    e_record, e_wait, e_sync, s_sync, sync = E.record, E.wait, E.synchronize, S.synchronize, torch.cuda.synchronize

    def record(self, stream=None):
        if T.active:
            T.record(self, _stream_ptr(stream))
        return e_record(self, stream)

    def wait(self, stream=None):
        if T.active:
            T.wait(self, _stream_ptr(stream))
        return e_wait(self, stream)

    def esync(self):
        if T.active and id(self) in T.ev:
            T.sync_clock(T.ev[id(self)])
        return e_sync(self)

    def ssync(self):
        if T.active:
            T.sync_clock(dict(T._clock(self.cuda_stream)))
        return s_sync(self)

    def dsync(device=None):
        if T.active:
            T.sync_all()
        return sync(device)

    E.record, E.wait, E.synchronize, S.synchronize, torch.cuda.synchronize = record, wait, esync, ssync, dsync
    # the step's device-scope link events (KDFM_LINK_EVENTS): the same edges
    L = K.LinkEvent
    l_record, l_wait = L.record, L.wait

    def lrecord(self, stream=None):
        if T.active:
            T.record(self, _stream_ptr(stream))
        return l_record(self, stream)

    def lwait(self, stream=None):
        if T.active:
            T.wait(self, _stream_ptr(stream))
        return l_wait(self, stream)

    L.record, L.wait = lrecord, lwait

    def all_reduce(tensor, op=None, group=None, async_op=False):
        s = _cur()
        T.pseudo += 1
        ps = f"collective#{T.pseudo}"
        T.vc[ps] = dict(T._clock(s))
        T.roles[ps] = "collective"
        sp = _span(tensor)
        if sp is not None:
            T.access(sp[0], sp[1], ps, True, _site(), "all_reduce")

        class Work:
            def wait(self_):
                T.sync_clock  # noqa: B018  (the waiting stream merges the collective's clock)
                v = T._clock(_cur())
                for k, c in T.vc[ps].items():
                    if v.get(k, 0) < c:
                        v[k] = c
                return True

        w = Work()
        if not async_op:
            w.wait()
            return None
        return w

    dist.all_reduce = all_reduce


def _on_call(name, args):
    from kdfm import kernels as K
    s = _cur()
    site = _site()
    if name in ("kdfm_event_record", "kdfm_stream_wait_event"):   # K.LinkEvent: ordering, hooked below
        return
    if name in ("kdfm_gemm", "kdfm_gemm_big", "kdfm_gemm_big_fp8"):
        v = K._GEMM_FMT.unpack_from(K._GEMM_BUF, 0)
        if name != "kdfm_gemm":   # its bf16 / fp8 operands and output are arguments; the descriptor carries the rest
            ops = ((args[1], "A16", 0), (args[3], "B16", 0), (args[6], "C16", 1)) if name == "kdfm_gemm_big" else \
                ((args[1], "A8", 0), (args[3], "B8", 0), (args[5], "sa", 0), (args[6], "sb", 0), (args[7], "C16", 1))
            for a, fld, w in ops:
                if a:
                    T.access(a, T.recent.get(a, a + 4), s, bool(w), site, f"gemm_big.{fld}")
        for idx, fld, w in ((0, "A", 0), (1, "B", 0), (2, "C", 1), (3, "bias", 0), (4, "R", 0), (5, "aux", 0),
                            (6, "Cpre", 1), (28, "seed", 0), (39, "mask_len", 0), (42, "loss_acc", 1),
                            (44, "ones_out", 1)):
            p = v[idx]
            if p:
                T.access(p, T.recent.get(p, p + 4), s, bool(w), site, f"gemm.{fld}")
        if v[46]:
            T.access(v[46], v[46] + 4 * v[47], s, True, site, "gemm.ws")
        return
    if name == "kdfm_wimg_prep_batch":
        for im in _imgsets():
            if im.table is not None and im.table.data_ptr() == args[0]:
                T.access(*_span(im.buf), s, True, site, "wimg.buf")
                for spec in im.specs:
                    for W in spec[6:8]:
                        if W is not None:
                            T.access(*_span(W), s, False, site, "wimg.W")
        return
    params = T.header.get(name)
    if params is None:
        return
    if name == "kdfm_ln_fold":
        n = int(args[3])
        for j, (pname, kind) in enumerate(params[:3]):
            arr = C.cast(args[j], C.POINTER(C.c_void_p))
            for i in range(n):
                p = arr[i]
                if p:
                    T.access(p, T.recent.get(p, p + 4), s, kind == "ww", site, f"{name}.{pname}[{i}]")
        return
    for (pname, kind), a in zip(params, args):
        if kind not in ("r", "w") or a is None:
            continue
        p = a.value if isinstance(a, C.c_void_p) else a
        if not isinstance(p, int) or p == 0:
            continue
        T.access(p, T.recent.get(p, p + 4), s, kind == "w", site, f"{name.replace('kdfm_', '')}.{pname}")


def _imgsets():
    from kdfm import kernels as K
    return [r() for r in K._IMGSETS if r() is not None]


_NOWRITE = {"empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "_local_scalar_dense",
            "record_stream", "set_", "resize_", "lift_fresh", "detach", "alias"}


class Mode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        if T is not None and T.active:
            try:
                _on_aten(func, args, kwargs, out)
            except Exception as e:  # the checker must never change the program
                print("race_check: aten hook failed on", func, e, file=sys.stderr)
        return out


def _on_aten(func, args, kwargs, out):
    base = func._schema.name.split("::")[-1]
    s = _cur()
    if base == "record_stream":
        T.record_stream(args[0].data_ptr(), _stream_ptr(args[1]))
        return
    if base == "_local_scalar_dense":
        if args[0].is_cuda:
            T.sync_clock(dict(T._clock(s)))
        return
    ins = []
    for i, a in enumerate(func._schema.arguments):
        val = args[i] if i < len(args) else kwargs.get(a.name)
        flat, _ = tree_flatten(val)
        for t in flat:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                ins.append((t, a.alias_info is not None and a.alias_info.is_write))
    outs = [t for t in tree_flatten(out)[0] if isinstance(t, torch.Tensor) and t.is_cuda]
    in_storages = {t.untyped_storage().data_ptr() for t, _ in ins}
    fresh = [t for t in outs if t.untyped_storage().data_ptr() not in in_storages]
    for t in fresh:
        st = t.untyped_storage()
        if st.nbytes():
            T.alloc(st.data_ptr(), st.data_ptr() + st.nbytes(), s)
    if base in _NOWRITE:
        return
    mutates = any(w for _, w in ins)
    if outs and not fresh and not mutates:
        return   # a view: no memory traffic
    site = _site()
    for t, w in ins:
        sp = _span(t)
        if sp:
            T.access(sp[0], sp[1], s, w, site, f"aten.{base}")
    for t in fresh:
        sp = _span(t)
        if sp:
            T.access(sp[0], sp[1], s, True, site, f"aten.{base}")


# ------------------------------------------------------------------------------------------------
# the scenario: the bench's overlapped bf16 step (+ the bucketed all-reduce of a world of 2)
# ------------------------------------------------------------------------------------------------

MUTATIONS = ("none", "heads_join", "bucket_early", "allreduce_caller")


def mutate(kind, eng):
    """Re-introduce an ordering defect into the step (checker self-test; the GPU then really runs the defect):
    * heads_join -- the first KD-heads half no longer joins the teacher stream before it reads the teacher
      features / auto-encoder outputs of layers [0, h) (the round-5 race, fixed in Ver5Engine._heads_first_half);
    * bucket_early -- the bucketed all-reduce launches every bucket at the backward's first gradient-ready point
      (after the KD heads), before the encoder layers' gradients are final: the collectives then read gradients
      the weight-gradient and compute streams still write (a collective issued ahead of its bucket's gradients).
      (Dropping only the weight-gradient stream's join with the compute stream before a bucket's collective is
      NOT a race here: every weight-gradient launch already joins it, the last one right before ready() --
      measured clean on the GPU, profiles/r06/r6a);
    * allreduce_caller -- the final all-reduce is called from the caller's stream instead of through
      Ver5Engine.allreduce_grads (the round-5 suspicion).  NOT a race by construction: backward() leaves the
      caller's stream waiting for the compute stream, so the checker must stay clean (a negative control)."""
    from kdfm.engine import Ver5Engine
    from kdfm.overlap import WGRAD
    if kind == "heads_join":
        orig = Ver5Engine._heads_first_half

        def heads_first_half(self, *a):
            from kdfm import kernels as K
            side = a[-1]
            ws_orig = K.wait_stream   # the engine's joins go through kernels.wait_stream (either link-event kind)

            def wait_stream(dst, src):
                if src.cuda_stream == side.cuda_stream:
                    return None   # the dropped join
                return ws_orig(dst, src)
            K.wait_stream = wait_stream
            try:
                return orig(self, *a)
            finally:
                K.wait_stream = ws_orig
        Ver5Engine._heads_first_half = heads_first_half
    elif kind == "bucket_early":
        from kdfm.ddp import BucketedGradAllReduce
        orig_ready = BucketedGradAllReduce.ready
        BucketedGradAllReduce.ready = lambda self, flat, offset: orig_ready(self, flat, 0)
    elif kind == "allreduce_caller":
        def allreduce_grads(self, allreduce):
            return allreduce(self.student.grad)
        eng.allreduce_grads = allreduce_grads.__get__(eng)
    elif kind != "none":
        raise ValueError(kind)


def run(layers=3, batch=8, seconds=16.0, steps=2, ddp=True, deterministic=False, math="bf16", verbose=True,
        diffkd=False, serial=False, mutation="none", plan=False):
    """serial: weight gradients and the first heads half in line (the deterministic schedule's stream structure
    without its ordered reductions); plan: the checked steps are a step plan's recording step (its host
    callbacks and launches as recorded) followed by eager steps."""
    from dataclasses import replace

    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.ddp import BucketedGradAllReduce
    from kdfm.engine import Ver5Engine, synthetic_batch
    from kdfm.overlap import WGRAD

    cfg = replace(DEFAULT, n_layers=layers, deterministic=deterministic, math=math, use_diffkd=diffkd)
    dev = torch.device("cuda", 0)
    tr = Tracer()
    install(tr)
    eng = Ver5Engine(cfg, dev)
    if serial:
        eng.overlap_wgrad = False
    mutate(mutation, eng)
    eng.set_seed(5)
    n = int(16000 * seconds)
    wav, wl, tg, tl = synthetic_batch(cfg, batch, n, 40, dev, seed=11)
    ar = None
    if ddp:
        dist.get_world_size = lambda group=None: 2
        ar = BucketedGradAllReduce(eng.student.numel, buckets=4)
    with Mode():
        eng.train_step(wav, wl, tg, tl, allreduce=ar)   # warm-up: lazily created streams / workspaces
        torch.cuda.synchronize()
        roles = {eng.compute_stream.cuda_stream: "compute", eng._side_stream().cuda_stream: "teacher",
                 eng._aux_stream().cuda_stream: "ctc_kl", 0: "null"}
        for k, st in WGRAD._side.items():
            roles[st.cuda_stream] = "wgrad"
        roles[torch.cuda.current_stream().cuda_stream] = roles.get(torch.cuda.current_stream().cuda_stream, "caller")
        tr.roles.update(roles)
        tr.active = True
        for i in range(steps):
            if plan and i == 0:
                eng.make_plan(wav, wl, tg, tl, ar)
            else:
                eng.train_step(wav, wl, tg, tl, allreduce=ar)
        tr.active = False
        torch.cuda.synchronize()
    if verbose:
        print(f"race_check: layers={layers} B={batch} {seconds}s steps={steps} ddp={ddp} math={math} "
              f"deterministic={deterministic} serial={eng._serial()} plan={plan} mutation={mutation} diffkd={diffkd} "
              f"heads_split={eng.heads_split}: {tr.naccess} accesses, {len(tr.vc)} streams, "
              f"{len(tr.conflicts)} conflicting site pairs")
    return tr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=16.0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--no-ddp", action="store_true")
    ap.add_argument("--math", default="bf16")
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--diffkd", action="store_true")
    ap.add_argument("--serial", action="store_true", help="weight gradients in line (overlap_wgrad=False)")
    ap.add_argument("--plan", action="store_true", help="the first checked step records a step plan")
    ap.add_argument("--mutate", default="none", choices=MUTATIONS, help="checker self-test: re-introduce a defect")
    a = ap.parse_args()
    tr = run(a.layers, a.batch, a.seconds, a.steps, not a.no_ddp, a.deterministic, a.math, diffkd=a.diffkd,
             serial=a.serial, mutation=a.mutate, plan=a.plan)
    n = tr.report()
    sys.exit(1 if n else 0)


if __name__ == "__main__":
    main()
