"""Step plans: record the training step's launch sequence once, replay it without the Python wrappers.

The step is issued eagerly on four HIP streams (compute, teacher, weight gradients, CTC/KL) and its
host-side enqueue -- ~1.2k libkdfm launches through typed Python wrappers, shape checks, tensor
allocations, stream switches -- costs ~13 ms against a ~19 ms GPU step.  A
captured HIP graph removes the host cost but on this ROCm loses the cross-stream overlap
(DESIGN.md §6).  A StepPlan keeps the eager multi-stream schedule and drops the Python:

  * record: one step runs normally while every libkdfm launch is captured as (ctypes function, the
    exact argument values, descriptor snapshots), every cross-stream edge as (event, stream) record /
    wait, and every host callback the step makes (the bucketed all-reduce's ready()) as a Python
    call; every tensor the step allocates is kept alive by the plan, so the recorded device
    addresses stay owned by it (the plan's private memory, like a graph pool);
  * replay: the same launches with the same arguments in the same order on the same streams,
    events re-recorded / waited through libkdfm's thin hipEventRecord / hipStreamWaitEvent wrappers.

Everything the step computes from changing state reads it on the device (RNG seed, step counter,
Noam learning rate, the inputs' static buffers), so a replay is the step.  The library's one
process-global launch setting, the deterministic-reduction mode (kdfm_set_deterministic: it picks
ordered or atomic reduction routes at launch time), is recorded with every launch and re-applied
around it on replay, so a plan recorded in deterministic mode replays the ordered kernels whatever
mode the caller is in.  Torch ops that touch
memory inside the recorded step are restricted to fills (replayed as kdfm_fill); anything else raises
at record time, so a plan is never silently incomplete.
"""
from __future__ import annotations

import ctypes as C
import os
import warnings

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from . import _lib
from . import kernels as K

_FILL_OPS = {"zeros", "zero_", "fill_", "ones", "full", "new_zeros"}
_NO_ACCESS = {"empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "record_stream", "detach",
              "alias", "lift_fresh", "_local_scalar_dense"}


class PlanError(RuntimeError):
    pass


# KDFM_PLAN_ELIDE=0: replay every recorded cross-stream link (A/B switch)
_ELIDE = os.environ.get("KDFM_PLAN_ELIDE", "1") == "1"


def _link(op):
    """("r" | "w", event handle, stream handle) of a link op (torch events "er" / "ew", or K.LinkEvent's
    kdfm_event_record / kdfm_stream_wait_event launches), else None."""
    if op[0] in ("er", "ew"):
        return op[0][1], op[1].value, op[2].value
    if op[0] == "k":
        nm = getattr(op[1], "__name__", "")
        if nm == "kdfm_event_record":
            return "r", op[2][0], op[2][1]
        if nm == "kdfm_stream_wait_event":
            return "w", op[2][1], op[2][0]
    return None


def _raw(v):
    return v.value if isinstance(v, C.c_void_p) else v


def _elide_links(ops):
    """Drop a link that repeats the previous one: an event re-recorded on stream S with nothing issued on S
    since its last record there, and the waits on it by streams that already waited on that earlier record
    (a wait binds to the latest record, which now marks the same point of S).  The recorded step makes these
    when two weight-gradient jobs fork off one compute-stream point; each record / wait is a packet on its
    stream's queue, between kernels.  Conservative: a launch is attributed to a stream only when one of its
    arguments is a stream the links use; a launch naming none of them, and a host callback, end every run."""
    streams = set()
    for op in ops:
        lk = _link(op)
        if lk is not None:
            streams.add(lk[2])
    out = []
    last = {}        # event -> (stream, ops issued on it up to and including the record, streams waited since)
    issued = {}      # stream -> ops issued on it so far
    dropped = set()  # events whose latest record was dropped
    for op in ops:
        lk = _link(op)
        if lk is None:
            hit = [a for a in (op[2] if op[0] == "k" else ()) if isinstance(a, (int, C.c_void_p)) and _raw(a) in streams]
            if not hit:
                last.clear()
                dropped.clear()
            for a in hit[-1:]:
                issued[_raw(a)] = issued.get(_raw(a), 0) + 1
            out.append(op)
            continue
        kind, ev, s = lk
        if kind == "r":
            prev = last.get(ev)
            if prev is not None and prev[0] == s and prev[1] == issued.get(s, 0):
                dropped.add(ev)   # the same point of s as the record the waiters already bound to
                continue
            dropped.discard(ev)
            issued[s] = issued.get(s, 0) + 1
            last[ev] = (s, issued[s], set())
            out.append(op)
        else:
            prev = last.get(ev)
            if ev in dropped and prev is not None and s in prev[2]:
                continue          # this stream already waits for that point
            if prev is not None:
                prev[2].add(s)
            issued[s] = issued.get(s, 0) + 1
            out.append(op)
    return out


class _Recorder(TorchDispatchMode):
    def __init__(self, plan):
        super().__init__()
        self.plan = plan

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        if self.plan._paused:
            return out
        name = func._schema.name.split("::")[-1]
        outs = [t for t in (out if isinstance(out, (tuple, list)) else (out,)) if isinstance(t, torch.Tensor)]
        ins = [a for a in args if isinstance(a, torch.Tensor)]
        for t in outs:
            self.plan.keep.append(t)
        if name in _NO_ACCESS:
            return out
        in_st = {t.untyped_storage().data_ptr() for t in ins}
        is_view = outs and all(t.untyped_storage().data_ptr() in in_st for t in outs) and not any(
            a.alias_info is not None and a.alias_info.is_write for a in func._schema.arguments)
        if is_view or not any(t.is_cuda for t in outs + ins):
            return out
        if name in _FILL_OPS:
            tgt = outs[0] if outs else args[0]
            val = 0.0
            if name in ("fill_", "full"):
                val = float(args[1])
            elif name == "ones":
                val = 1.0
            if not tgt.is_contiguous():
                self.plan._bad.append(f"{func} on a non-contiguous tensor")
            elif val == 0.0:   # zero fill of any dtype: a memset of its bytes
                self.plan.ops.append(("k", self.plan._fn("kdfm_memset_async"),
                                      (tgt.data_ptr(), 0, tgt.numel() * tgt.element_size(), K.stream_ptr()),
                                      K.get_deterministic()))
            elif tgt.dtype == torch.float32:
                self.plan.ops.append(("k", self.plan._fn("kdfm_fill"), (tgt.data_ptr(), val, tgt.numel(),
                                                                        K.stream_ptr()), K.get_deterministic()))
            else:
                self.plan._bad.append(f"{func} = {val} on {tgt.dtype}")
            return out
        self.plan._bad.append(str(func))
        return out


class StepPlan:
    """Record `fn()` (one training step, device work only) once; `replay()` re-issues it."""

    def __init__(self):
        self.ops = []      # ("k", ctypes fn, args, det) | ("er", event, stream) | ("ew", event, stream) | ("py", fn, args)
        self.keep = []     # every tensor / event / descriptor the recorded launches address
        self._bad = []
        self._paused = False
        self._fns = {}
        lib = _lib.lib()
        self._ev_record = lib.kdfm_event_record
        self._ev_wait = lib.kdfm_stream_wait_event

    def _fn(self, name):
        f = self._fns.get(name)
        if f is None:
            f = self._fns[name] = getattr(_lib.lib(), name)
        return f

    # ---- recording ----------------------------------------------------------------------------
    def host(self, fn, *args):
        """Run a host callback now and replay it in place (e.g. the bucketed all-reduce's ready()):
        whatever it issues is not recorded, it is re-issued by the callback on every replay."""
        self.ops.append(("py", fn, args))
        self._paused = True
        try:
            fn(*args)
        finally:
            self._paused = False

    def record(self, fn):
        plan = self
        orig_call = K.call
        E = torch.cuda.Event
        e_record, e_wait = E.record, E.wait

        def call(name, *args):
            orig_call(name, *args)
            if plan._paused:
                return
            if name in ("kdfm_gemm", "kdfm_gemm_big", "kdfm_gemm_big_fp8"):   # the descriptor buffer is shared by every launch: snapshot it
                buf = C.create_string_buffer(K._GEMM_BUF.raw, len(K._GEMM_BUF.raw))
                plan.keep.append(buf)
                args = (C.cast(buf, C.POINTER(_lib.GemmDesc)),) + tuple(args[1:])
            plan.keep.append(args)
            plan.ops.append(("k", plan._fn(name), args, K.get_deterministic()))

        def record_ev(self_ev, stream=None):
            e_record(self_ev, stream)
            if not plan._paused:
                s = stream.cuda_stream if stream is not None else K.stream_ptr()
                plan.keep.append(self_ev)
                plan.ops.append(("er", self_ev, s))

        def wait_ev(self_ev, stream=None):
            e_wait(self_ev, stream)
            if not plan._paused:
                s = stream.cuda_stream if stream is not None else K.stream_ptr()
                plan.keep.append(self_ev)
                plan.ops.append(("ew", self_ev, s))

        K.call, E.record, E.wait = call, record_ev, wait_ev
        try:
            with _Recorder(self):
                fn()
        finally:
            K.call, E.record, E.wait = orig_call, e_record, e_wait
        if self._bad:
            raise PlanError(f"the step issues torch ops a plan cannot replay: {sorted(set(self._bad))[:8]}")
        # resolve the raw event handles once (events exist after their first record)
        ops = []
        # KDFM_PLAN_KNOCKOUT=name[,name...]: drop those entries' launches from the replay -- a what-if probe
        # of a kernel family's share of the step (tools/runs/knockout); the replayed step's results are wrong
        knock = {n for n in os.environ.get("KDFM_PLAN_KNOCKOUT", "").split(",") if n}
        if knock:
            warnings.warn(f"KDFM_PLAN_KNOCKOUT={sorted(knock)}: the replayed step skips these launches (probe only)")
        for op in self.ops:
            if op[0] == "k" and knock and op[1].__name__ in knock:
                continue
            if op[0] in ("er", "ew"):
                ops.append((op[0], C.c_void_p(op[1].cuda_event), C.c_void_p(op[2])))
            else:
                ops.append(op)
        self.ops = _elide_links(ops) if _ELIDE else ops
        return self

    # ---- replay ---------------------------------------------------------------------------------
    def replay(self):
        rec, wt = self._ev_record, self._ev_wait
        saved = K.get_deterministic()
        det = saved
        try:
            for op in self.ops:
                kind = op[0]
                if kind == "k":
                    if op[3] != det:
                        det = op[3]
                        K.set_deterministic(det)
                    rc = op[1](*op[2])
                    if rc:
                        _lib.check(rc, "plan replay")
                elif kind == "er":
                    rc = rec(op[1], op[2])
                    if rc:
                        _lib.check(rc, "plan replay (event record)")
                elif kind == "ew":
                    rc = wt(op[2], op[1])
                    if rc:
                        _lib.check(rc, "plan replay (stream wait)")
                else:
                    op[1](*op[2])
        finally:
            if det != saved:
                K.set_deterministic(saved)

    def __len__(self):
        return len(self.ops)


__all__ = ["StepPlan", "PlanError"]
