"""Thin, typed Python wrappers over the libkdfm.so C-ABI (no autograd here).

Tensors are torch CUDA tensors used purely as device allocations (the caching allocator owns the
memory, torch's current HIP stream orders the work); every arithmetic operation runs in a libkdfm
kernel.  Each wrapper validates shapes on the host before the launch, so a bad call raises here
instead of faulting on the device.
"""
from __future__ import annotations

import ctypes as C
import os
import struct

import torch

from . import _lib
from ._lib import GemmDesc, call

_MATH = {"f32": _lib.KDFM_MATH_F32, "bf16": _lib.KDFM_MATH_BF16}


class _State:
    math = "f32"
    deterministic = False
    fp8 = False   # the large-tile route's forward / data-gradient products in fp8 e4m3 (Ver5Config.linear_fp8)
    # weight epoch: while set (the engine advances it once per step, before the forward), each weight's bf16 copy of
    # the large-tile route and its MX fp8 copies are made at its first use in the epoch and reused after; None
    # (the module API, tests): every product converts its weight itself
    ranges = os.environ.get("KDFM_ROCTX", "0") == "1"   # ROCTx ranges around engine phases


ROUTES = {0: "generic", 1: "skinny", 2: "rowstream_fwd", 3: "wide_wgrad", 4: "split_fold", 5: "slab_conv",
          6: "wgrad_rows", 7: "big"}


class Trace:
    """Brackets launches with HIP events on the launch stream (bench.py's live per-kernel timing):
    every GEMM launch carrying one of `tags` (tag "*" = every kdfm_gemm call; those are also keyed
    by the kernel family libkdfm routed them to, kdfm_gemm_last_route), and every `span(tag)` block.
    Each record carries the algorithmic FLOPs and HBM bytes of the launch."""
    active = None

    def __init__(self, tags):
        self.tags = set(tags)
        self.events = []   # (tag, flops, algorithmic bytes, start, end, raw stream)

    def __enter__(self):
        Trace.active = self
        return self

    def __exit__(self, *a):
        Trace.active = None

    def wants(self, tag):
        return tag in self.tags or ("*" in self.tags and tag is None)

    def summary(self, stream=None):
        """{tag: launches, ms_total, flops_total, bytes_total}; with `stream` (a raw stream pointer)
        only the launches issued on that stream (e.g. the engine's critical-path compute stream)."""
        torch.cuda.synchronize()
        out = {}
        for tag, flops, nbytes, s, e, st in self.events:
            if stream is not None and st != stream:
                continue
            ms = s.elapsed_time(e)
            t = out.setdefault(tag, [0, 0.0, 0.0, 0.0])
            t[0] += 1
            t[1] += ms
            t[2] += flops
            t[3] += nbytes
        return {k: {"launches": v[0], "ms_total": v[1], "flops_total": v[2], "bytes_total": v[3]}
                for k, v in out.items()}


def _traced(tag, flops, nbytes, name, *args):
    """call(name, *args); when the active Trace wants `tag` (or "*"), bracket the launch with HIP events
    on the current stream and record its algorithmic FLOPs / HBM bytes (bench.py roofline families)."""
    tr = Trace.active
    if tr is None or not (tag in tr.tags or "*" in tr.tags):
        call(name, *args)
        return
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    call(name, *args)
    ev1.record()
    tr.events.append((tag, float(flops), float(nbytes), ev0, ev1, stream_ptr()))


def set_ranges(on: bool) -> None:
    """Emit ROCTx ranges (kdfm_range_push/pop) around the engine's phases and every span(); env
    KDFM_ROCTX=1 sets it at import.  rocprofv3 --marker-trace records them with the kernels."""
    _State.ranges = bool(on)


class region:
    """Context manager: one ROCTx range named `name` on this host thread when ranges are on."""
    __slots__ = ("name", "on")

    def __init__(self, name):
        self.name = name
        self.on = False

    def __enter__(self):
        if _State.ranges:
            _lib.lib().kdfm_range_push(("kdfm:" + self.name).encode())
            self.on = True
        return self

    def __exit__(self, *a):
        if self.on:
            _lib.lib().kdfm_range_pop()


class span(region):
    """Context manager: time the enclosed launches (one stream) as one record of `tag` when the
    active Trace asks for it (and a ROCTx range of the same name when ranges are on)."""
    __slots__ = ("tag", "nbytes", "flops", "ev")

    def __init__(self, tag, nbytes=0.0, flops=0.0):
        super().__init__(tag)
        self.tag, self.nbytes, self.flops = tag, nbytes, flops
        self.ev = None

    def __enter__(self):
        super().__enter__()
        tr = Trace.active
        if tr is not None and self.tag in tr.tags:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        return self

    def __exit__(self, *a):
        if self.ev is not None:
            self.ev[1].record()
            Trace.active.events.append((self.tag, self.flops, self.nbytes, self.ev[0], self.ev[1], stream_ptr()))
        super().__exit__(*a)


def set_math(mode: str) -> None:
    if mode not in _MATH:
        raise ValueError(f"math mode must be one of {list(_MATH)}")
    _State.math = mode


def get_math() -> str:
    return _State.math


def set_deterministic(on: bool) -> None:
    """Deterministic-reduction mode of the library (include/kdfm.h kdfm_set_deterministic): ordered
    reductions everywhere an activation or gradient is summed, bitwise reproducible runs."""
    _lib.lib().kdfm_set_deterministic(1 if on else 0)
    _State.deterministic = bool(on)


def get_deterministic() -> bool:
    return _State.deterministic


class mode:
    """Context manager: run a block in the given MFMA arithmetic / reduction mode and restore the
    previous process-global modes afterwards (the engine applies its config this way)."""

    def __init__(self, math: str | None = None, deterministic: bool | None = None, fp8: bool | None = None,
                 wide: bool | None = None):
        self.math, self.det, self.fp8, self.wide = math, deterministic, fp8, wide

    def __enter__(self):
        self._saved = (_State.math, _State.deterministic, _State.fp8, _State.wide)
        if self.math is not None:
            set_math(self.math)
        if self.det is not None and self.det != _State.deterministic:
            set_deterministic(self.det)
        if self.fp8 is not None:
            _State.fp8 = bool(self.fp8)
        if self.wide is not None:
            _State.wide = bool(self.wide)
        return self

    def __exit__(self, *a):
        m, d, f8, w = self._saved
        set_math(m)
        if d != _State.deterministic:
            set_deterministic(d)
        _State.fp8 = f8
        _State.wide = w


def set_wide(on: bool) -> None:
    """Wide-model routing (d_model >= 512): the large-tile route also takes products with a dimension in
    [64, 512) when another is >= 1024 (big_ok).  Process-global like the math mode; the engine sets it from
    its config for the duration of a call."""
    _State.wide = bool(on)


def set_fp8(on: bool) -> None:
    """fp8 e4m3 operands (MX block scaling) for the large-tile route's forward and data-gradient products
    (kdfm_gemm_big_fp8); weight gradients stay bf16.  Process-global like the math mode."""
    _State.fp8 = bool(on)


def get_fp8() -> bool:
    return _State.fp8


_State.fp8_epoch = None
_State.wide = False
_FP8_W = {}   # (address, rows, cols, row stride, transposed) -> [epoch, storage, (address, ld, scales)]
_BF16_W = {}  # (address, rows, cols, row stride) -> [epoch, bf16 storage]


_EPOCHS = [0]


class weight_epoch:
    """Context manager (the engine wraps each forward / backward / inference call in one): inside it, the weights
    are constant, so the large-tile route converts each weight (bf16, MX fp8) once at its first use and reuses the
    copy; outside (the module API, tests, after an optimizer step) every product converts its weight itself."""

    def __enter__(self):
        # nested inside an open epoch (the engine's train_step around its forward and backward): join it -- the
        # weights cannot change before the outer one closes, so the backward reuses the forward's copies
        self._saved = _State.fp8_epoch
        if self._saved is None:
            _EPOCHS[0] += 1
            _State.fp8_epoch = _EPOCHS[0]
        return self

    def __exit__(self, *a):
        _State.fp8_epoch = self._saved


_FROZEN = []   # (first byte, end byte, weakref to the owner with .version, token): frozen parameter buffers
_FROZEN_TOKENS = [0]


def register_frozen(buf, owner) -> None:
    """Declare `buf`'s parameters frozen (the distillation teacher): the large-tile route's bf16 / MX copies of its
    weight views are made once and reused across engine calls until `owner.version` changes (FlatStore.load bumps
    it).  A step plan recorded after the copies exist replays no conversion for them: reload the teacher before
    recording plans.  Each registration has its own token, so a later buffer at the same address never matches an
    earlier one's copies; dead owners' entries (and their copies) are dropped here."""
    import weakref
    dead = [f for f in _FROZEN if f[2]() is None]
    for lo, hi, _, _ in dead:
        for cache in (_BF16_W, _FP8_W):
            for k in [k for k in cache if lo <= k[0] < hi]:
                del cache[k]
    lo = buf.data_ptr()
    _FROZEN[:] = [f for f in _FROZEN if f[2]() is not None and f[0] != lo]
    _FROZEN_TOKENS[0] += 1
    _FROZEN.append((lo, lo + buf.numel() * buf.element_size(), weakref.ref(owner), _FROZEN_TOKENS[0]))


def _epoch_of(W):
    """The cache tag a weight view's converted copy is valid for: the owner's version for a frozen buffer, else
    the current engine-call epoch (None outside one: convert per use)."""
    p = W.data_ptr()
    for lo, hi, ref, tok in _FROZEN:
        if lo <= p < hi:
            owner = ref()
            if owner is not None:
                return ("frozen", tok, owner.version)
    return _State.fp8_epoch


_MIRRORS = []   # (first byte, end byte, bf16 mirror tensor): flat parameter buffers with a maintained bf16 mirror


def register_bf16_mirror(buf, mirror) -> None:
    """`mirror` (bf16, same element layout) is kept equal to bf16(buf) by its owner (FlatStore: refreshed on load,
    written by AdamW in the same pass, kdfm_adamw_noam_bf16): the large-tile route reads weight views of `buf` from
    it directly -- no cast per engine call."""
    lo = buf.data_ptr()
    _MIRRORS[:] = [m for m in _MIRRORS if m[0] != lo]
    _MIRRORS.append((lo, lo + buf.numel() * 4, mirror))


def _mirror_of(W):
    p = W.data_ptr()
    for lo, hi, mir in _MIRRORS:
        if lo <= p < hi and W.dtype == torch.float32 and W.stride(1) == 1 and W.stride(0) % 8 == 0:
            a = mir.data_ptr() + (p - lo) // 2
            if a % 16 == 0:
                return a, W.stride(0)
    return None


def _bf16_weight(W):
    """The large-tile route's bf16 copy of a weight view for this epoch (cast on first use), or None outside an
    epoch; persistent storage (a recorded plan replays the cast into it).  Frozen weights: once per version.  A
    weight inside a mirrored flat buffer (register_bf16_mirror): its mirror view, no copy."""
    m = _mirror_of(W)
    if m is not None:
        return m
    ep = _epoch_of(W)
    if ep is None or W.dtype != torch.float32:
        return None
    key = (W.data_ptr(), W.shape[0], W.shape[1], W.stride(0))
    ent = _BF16_W.get(key)
    ld = -(-W.shape[1] // 8) * 8
    if ent is None:
        ent = _BF16_W[key] = [None, torch.empty(W.shape[0], ld, dtype=torch.bfloat16, device=W.device)]
    if ent[0] != ep:
        call("kdfm_cast_bf16_2d", ptr(W), W.stride(0), ent[1].data_ptr(), ld, W.shape[0], W.shape[1], _s())
        ent[0] = ep
    return ent[1].data_ptr(), ld


def _fp8_weight(W, tr):
    """The MX copy of a weight view for this epoch (quantised on first use; kdfm_fp8_quant_mx), or None outside an
    epoch.  The copies are persistent (a recorded step plan replays the quantisation launch into the same storage).
    Frozen weights (register_frozen): once per version."""
    ep = _epoch_of(W)
    if ep is None:
        return None
    key = (W.data_ptr(), W.shape[0], W.shape[1], W.stride(0), bool(tr))
    ent = _FP8_W.get(key)
    r, kc = (W.shape[1], W.shape[0]) if tr else (W.shape[0], W.shape[1])
    ld = -(-kc // 16) * 16
    if ent is None:
        buf = torch.empty(r * ld + -(-(r * kc // 32) // 16) * 16, dtype=torch.uint8, device=W.device)
        ent = _FP8_W[key] = [None, buf, (buf.data_ptr(), ld, buf.data_ptr() + r * ld)]
    if ent[0] != ep:
        a, ld_, sc = ent[2]
        call("kdfm_fp8_quant_mx", ptr(_f32(W)), 0, W.shape[0], W.shape[1], W.stride(0), a, ld_, sc, 1 if tr else 0,
             _s())
        ent[0] = ep
    return ent[2]


# host-issue fast paths: torch.cuda.current_stream() costs several µs per call in Python (device
# index resolution, availability checks, a Stream object); the enqueue of one step makes ~1.3k of
# these queries, so the raw C entry points are used directly
_cur_dev = torch._C._cuda_getDevice
_raw_stream = torch._C._cuda_getCurrentRawStream


def stream_ptr() -> int:
    return _raw_stream(_cur_dev())


def current_device() -> int:
    return _cur_dev()


class on_stream:
    """torch.cuda.stream(s) without the Python overhead: makes `s` (a torch.cuda.Stream on the current
    device) torch's current stream for the block and restores the previous one afterwards."""
    __slots__ = ("s", "prev")

    def __init__(self, s):
        self.s = s

    def __enter__(self):
        s = self.s
        self.prev = torch._C._cuda_getCurrentStream(s.device_index)
        torch._C._cuda_setStream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *a):
        p = self.prev
        torch._C._cuda_setStream(stream_id=p[0], device_index=p[1], device_type=p[2])


# Release scope of the step's cross-stream link events (KDFM_LINK_EVENTS): "nofence" (default) =
# hipEventDisableSystemFence, "device" = hipEventReleaseToDevice, "system" = torch.cuda.Event (HIP's default
# system-scope fence on every record).  Every link joins two streams of ONE device, whose kernels already see
# each other's writes at the device-scope release / acquire every kernel boundary has, and no link event is
# ever host-synchronised or queried.  Measured (profiles/r06/r6ar): nofence 2437 / 2441 utt/s against 2402 /
# 2405 (system) and 2403 / 2401 (device), interleaved on one box.
_LINK_FLAGS = {"system": None, "device": 0x40000000, "nofence": 0x20000000}[
    __import__("os").environ.get("KDFM_LINK_EVENTS", "nofence")]


class LinkEvent:
    """A hipEvent_t made by kdfm_event_create with the link flags; record / wait go through `call`, so a step
    plan records and replays them like launches."""
    __slots__ = ("cuda_event", "__weakref__")

    def __init__(self, flags):
        h = C.c_void_p()
        _lib.check(_lib.lib().kdfm_event_create(C.byref(h), flags), "kdfm_event_create")
        self.cuda_event = h.value

    def record(self, stream=None):
        call("kdfm_event_record", self.cuda_event, stream.cuda_stream if stream is not None else stream_ptr())

    def wait(self, stream=None):
        call("kdfm_stream_wait_event", stream.cuda_stream if stream is not None else stream_ptr(), self.cuda_event)

    def __del__(self):
        try:
            _lib.lib().kdfm_event_destroy(self.cuda_event)
        except Exception:   # interpreter shutdown
            pass


def link_event():
    return torch.cuda.Event() if _LINK_FLAGS is None else LinkEvent(_LINK_FLAGS)


class StreamLink:
    """Cross-stream ordering with one reusable event (a stream wait binds to the record made before
    it, so re-recording later is safe): `after_current(dst)` makes dst wait for the current stream,
    `current_after(src)` makes the current stream wait for src."""
    __slots__ = ("ev",)

    def __init__(self):
        self.ev = None

    def _event(self):
        if self.ev is None:
            self.ev = link_event()
        return self.ev

    def after_current(self, dst):
        ev = self._event()
        ev.record()
        ev.wait(dst)

    def current_after(self, src):
        ev = self._event()
        ev.record(src)
        ev.wait()


_WAIT_LINKS = {}


def wait_stream(dst, src):
    """dst.wait_stream(src) through a reusable link event per (dst, src) pair (torch's wait_stream makes a new
    system-scope event every call)."""
    if _LINK_FLAGS is None:
        dst.wait_stream(src)
        return
    key = (dst.cuda_stream, src.cuda_stream)
    ev = _WAIT_LINKS.get(key)
    if ev is None:
        ev = _WAIT_LINKS[key] = LinkEvent(_LINK_FLAGS)
    ev.record(src)
    ev.wait(dst)


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.KdfmError("kdfm kernels need device tensors (HIP); got a CPU tensor")
    return t.data_ptr()


def _f32(t, name="tensor"):
    if t is not None and t.dtype != torch.float32:
        raise _lib.KdfmError(f"{name} must be float32, got {t.dtype}")
    return t


def _i64(t, name="lengths"):
    if t is not None and t.dtype != torch.int64:
        raise _lib.KdfmError(f"{name} must be int64, got {t.dtype}")
    return t


def _s():
    return stream_ptr()


_SCRATCH: dict = {}
_RETIRED: list = []


def scratch(dev, nfloats: int, slot: int = 0):
    """f32 scratch for per-block reduction partials, one buffer per (device, stream, slot).  Consumers
    use it strictly in stream order (kernel then fold), so one buffer serves every call site of a
    stream (the weight-gradient side stream gets its own); it only grows.  Slot 1: a second buffer for a
    launch that needs two at once (the large-tile route's bf16 operand copies in slot 0, its split partials)."""
    import os
    idx = torch.device(dev).index if torch.device(dev).index is not None else torch.cuda.current_device()
    key = (idx, _raw_stream(idx)) if slot == 0 else (idx, _raw_stream(idx), slot)
    buf = _SCRATCH.get(key)
    if buf is None or buf.numel() < nfloats:
        if buf is not None and os.environ.get("KDFM_SCRATCH_RETIRE", "1") == "1":
            _RETIRED.append(buf)
        buf = torch.empty(max(int(nfloats), 1 << 16), device=dev, dtype=torch.float32)
        _SCRATCH[key] = buf
    return buf


# ------------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------------

# ------------------------------------------------------------------------------------------------
# bf16 weight twins (kdfm_gemm_desc.Bh): an f32 parameter buffer registered here has a bf16 copy
# in the same layout (forward products read W[n][k] rows) and, for every 2-D weight, a transposed
# copy at the same offset (data-gradient products read W^T rows).  The owner refreshes them with
# cast_bf16 / cast_bf16_t whenever the f32 values change (the engine: at the top of every step).
# ------------------------------------------------------------------------------------------------

class _Twin:
    def __init__(self, src, h, ht, entries):
        import weakref
        self.src = weakref.ref(src)
        self.base = src.data_ptr()
        self.end = self.base + 4 * src.numel()
        self.h, self.ht = h, ht
        self.entries = sorted(entries)              # (offset, rows, cols) of the transposed images
        self.starts = [e[0] for e in self.entries]


_TWINS: list = []


def twins_enabled() -> bool:
    """The direct-B skinny path that reads the twins is opt-in (KDFM_SKINNY_DIRECT_MIN_M)."""
    import os
    return bool(os.environ.get("KDFM_SKINNY_DIRECT_MIN_M"))


def register_bf16_twin(src, h, ht=None, entries=()):
    """src: f32 flat buffer; h: bf16 copy (same numel); ht: bf16 per-entry transposes or None."""
    assert src.dtype == torch.float32 and h.dtype == torch.bfloat16 and h.numel() == src.numel()
    _TWINS[:] = [t for t in _TWINS if t.src() is not None]
    _TWINS.append(_Twin(src, h, ht, entries))


def bf16_twin(W, transposed=False):
    """(device pointer, row stride) of the bf16 twin of weight view W — rows = W's rows (forward,
    B(k,n) = W[n][k]) or W's columns (transposed: B(k,n) = W[k][n]) — or None."""
    import bisect
    if W.dim() != 2 or W.stride(1) != 1:
        return None
    p = W.data_ptr()
    for t in _TWINS:
        if not (t.base <= p < t.end) or t.src() is None:
            continue
        off = (p - t.base) // 4
        if not transposed:
            return t.h.data_ptr() + 2 * off, W.stride(0)
        if t.ht is None:
            return None
        i = bisect.bisect_right(t.starts, off) - 1
        if i < 0:
            return None
        eoff, rows, cols = t.entries[i]
        rel = off - eoff
        r0, c0 = divmod(rel, cols)
        if rel >= rows * cols or W.stride(0) != cols or r0 + W.shape[0] > rows or c0 + W.shape[1] > cols:
            return None
        return t.ht.data_ptr() + 2 * (eoff + c0 * rows + r0), rows
    return None


def cast_bf16(src, dst):
    assert src.is_contiguous() and dst.is_contiguous() and src.numel() == dst.numel()
    call("kdfm_cast_bf16", ptr(_f32(src)), ptr(dst), src.numel(), _s())


def cast_bf16_t(src, dst, table, ntab, nblocks):
    call("kdfm_cast_bf16_t", ptr(_f32(src)), ptr(dst), ptr(table), int(ntab), int(nblocks), _s())


# kdfm_gemm_desc packed with one struct call into a reusable buffer (filling a ctypes Structure
# field by field cost ~6 µs of host time per GEMM launch).  Field order / native alignment match
# include/kdfm.h kdfm_gemm_desc (tests/test_abi.py checks the layout against GemmDesc).  Launches are
# issued from one host thread (the engine's), so one buffer suffices.
_GEMM_FMT = struct.Struct("@7P17q4fPQ7i2qPqqPfPqPqPq")
_GEMM_BUF = C.create_string_buffer(_GEMM_FMT.size)
_GEMM_DESC = C.cast(_GEMM_BUF, C.POINTER(GemmDesc))
_GEMM_WS_OFF = _GEMM_FMT.size - 4 * 8   # (ws, ws_len, Bh, sBh) are the last four 8-byte fields


def _p(t):
    return 0 if t is None else ptr(t)


def gemm(A, B, Cout, M, N, K, sAm, sAk, sBk, sBn, sCm, sCn, *, amode, bmode,
         batch=(1, 1), bA=(0, 0), bB=(0, 0), bC=(0, 0), alpha=1.0, epi=0, bias=None, R=None, rscale=1.0,
         aux=None, Cpre=None, beta=0.0, dropout_p=0.0, seed=None, rng_stream=0, splitk=1,
         conv=None, math=None, rowmask=None, mse=None, tag=None, ones_out=None, Bh=None, nbytes=None, big=None,
         fp8=None):
    """big = (A16 address, lda, B16 address, ldb, layout, C16 address or 0): the descriptor's epilogue on the
    large-tile bf16 kernel (kdfm_gemm_big) instead of kdfm_gemm's routes (see _big_linear)."""
    mth = math or _State.math
    bh, sbh = Bh if (Bh is not None and mth == "bf16") else (None, 0)
    ones_col = int(N) - 1 if ones_out is not None else -1
    if dropout_p > 0.0:
        epi |= _lib.EPI_DROPOUT
    taps, pad, cc, ct = conv if conv is not None else (0, 0, 0, 0)
    mlen, mT, mdiv = 0, 0, 0
    if rowmask is not None:
        lens, mT, mdiv = rowmask
        mlen = ptr(_i64(lens))
        epi |= _lib.EPI_ROWMASK
    lacc, lscale = 0, 0.0
    if mse is not None:
        acc, lscale = mse
        lacc = ptr(acc)
        epi |= _lib.EPI_MSE
    math_id = _MATH[mth]
    vals = [ptr(A), ptr(B), ptr(Cout), _p(bias), _p(R), _p(aux), _p(Cpre),
            int(M), int(N), int(K), sAm, sAk, sBk, sBn, sCm, sCn, batch[0], batch[1],
            bA[0], bA[1], bB[0], bB[1], bC[0], bC[1],
            alpha, beta, rscale, dropout_p, _p(seed), rng_stream,
            amode, bmode, epi, math_id, splitk, taps, pad, cc, ct,
            mlen, int(mT), int(mdiv), lacc, float(lscale), _p(ones_out), ones_col,
            0, 0, bh or 0, sbh]   # Bh: (device address, row stride) of the bf16 twin
    _GEMM_FMT.pack_into(_GEMM_BUF, 0, *vals)
    if fp8 is not None:   # (A8, lda, B8, ldb, A scales, B scales, C16): kdfm_gemm_big_fp8
        name, args = "kdfm_gemm_big_fp8", (_GEMM_DESC,) + tuple(fp8) + (_s(),)
    elif big is not None:
        name, args = "kdfm_gemm_big", (_GEMM_DESC,) + tuple(big) + (_s(),)
        if big[4] == _lib.BIG_TN:   # split-reduction partials (deterministic fold), when the shape asks for them
            nws = _lib.lib().kdfm_gemm_big_ws(int(M), int(N), int(K), int(big[4]))
            if nws > 0:
                ws = scratch(Cout.device, nws, slot=1)
                struct.pack_into("@Pq", _GEMM_BUF, _GEMM_WS_OFF, ws.data_ptr(), ws.numel())
    else:
        name, args = "kdfm_gemm", (_GEMM_DESC, _s())
    if big is None and fp8 is None and epi == _lib.EPI_ATOMIC and (math_id == _lib.KDFM_MATH_BF16 or (_State.deterministic and splitk > 1)):
        nws = _lib.lib().kdfm_gemm_ws(_GEMM_DESC)
        if nws > 0:
            ws = scratch(Cout.device, nws)
            struct.pack_into("@Pq", _GEMM_BUF, _GEMM_WS_OFF, ws.data_ptr(), ws.numel())
    tr = Trace.active
    if tr is not None and (tag in tr.tags or "*" in tr.tags):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        call(name, *args)
        ev1.record()
        if nbytes is None:   # fp32 storage: both operands and the output once, plus each side operand
            side = sum(1 for t in (R, aux, Cpre) if t is not None)
            nbytes = 4.0 * (M * K + K * N + M * N * (1 + side)) * batch[0] * batch[1]
        fl = 2.0 * M * N * K * batch[0] * batch[1]
        sp = stream_ptr()
        if tag in tr.tags:
            tr.events.append((tag, fl, nbytes, ev0, ev1, sp))
        if "*" in tr.tags:
            tr.events.append(("gemm:" + ROUTES.get(int(_lib.lib().kdfm_gemm_last_route()), "?"), fl, nbytes, ev0, ev1,
                              sp))
        return
    call(name, *args)


# ------------------------------------------------------------------------------------------------
# Large-tile bf16 route (csrc/biggemm.hip, kdfm_gemm_big) for the wide layer products (d_model >= 512:
# Conformer-large, FastConformer(-XL)).  Operands are bf16 in HBM: a bf16 tensor is read in place, an f32 one is
# cast into this stream's scratch first (kdfm_cast_bf16_2d); a bf16 `out` receives the product in bf16 (what the
# next product reads: the FFN hidden activation and its gradient), which only this route can write.
# KDFM_BIG_GEMM=0: the kdfm_gemm routes (f32 operands only).
# ------------------------------------------------------------------------------------------------
_BIG = os.environ.get("KDFM_BIG_GEMM", "1") == "1"
_BIG_MIN_WORK = float(os.environ.get("KDFM_BIG_MIN_WORK", str(2 ** 31)))   # M * N * K


def big_ok(M, N, K, layout) -> bool:
    """The large-tile route takes this product (bf16 math, M * N * K >= 2^31, every dimension >= 512 -- or, in
    the wide-model mode (set_wide: d_model >= 512, the engine's config), every dimension >= 64 and one >= 1024:
    FastConformer-XL's 256-channel pointwise subsampling convs and its d -> 1024 distillation-head projections)."""
    if not _BIG or _State.math != "bf16" or float(M) * N * K < _BIG_MIN_WORK:
        return False
    lo = min(M, N, K)
    if lo < 512 and not (_State.wide and lo >= 64 and max(M, N, K) >= 1024):
        return False
    return bool(_lib.lib().kdfm_gemm_big_supported(int(M), int(N), int(K), int(layout)))


def _bf16_operands(ts, weight=None):
    """(address, row stride) of each 2-D operand as bf16: bf16 tensors in place, f32 ones cast into scratch; index
    `weight` names a weight view, whose per-epoch copy (_bf16_weight) is used when there is one."""
    wcopy = _bf16_weight(ts[weight]) if weight is not None else None
    if wcopy is not None:
        rest = _bf16_operands([t for i, t in enumerate(ts) if i != weight])
        rest.insert(weight, wcopy)
        return rest
    need = []
    for t in ts:
        if t.dtype == torch.bfloat16:
            assert t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0, "bf16 operand layout"
        else:
            _f32(t)
            need.append(t)
    out = []
    if need:
        sizes = [(t.shape[0] * (-(-t.shape[1] // 8) * 8)) for t in need]
        buf = scratch(need[0].device, (sum(sizes) + 8 * len(sizes)) // 2 + 8).view(torch.bfloat16)
        off = 0
        cast = {}
        for t, n in zip(need, sizes):
            ld = -(-t.shape[1] // 8) * 8
            dst = buf.data_ptr() + 2 * off
            call("kdfm_cast_bf16_2d", ptr(t), t.stride(0), dst, ld, t.shape[0], t.shape[1], _s())
            cast[id(t)] = (dst, ld)
            off += n
    for t in ts:
        out.append((t.data_ptr(), t.stride(0)) if t.dtype == torch.bfloat16 else cast[id(t)])
    return out


def fp8_ok(M, N, K) -> bool:
    """The fp8 instance takes this k-contiguous product (fp8 mode on, the large-tile route applies, K % 128 == 0,
    M and N multiples of 4, every dimension >= 512: the layer Linears; the wide-model mode's narrower products
    (set_wide) stay bf16)."""
    return (_State.fp8 and K % 128 == 0 and M % 4 == 0 and N % 4 == 0 and min(M, N, K) >= 512
            and big_ok(M, N, K, _lib.BIG_NT))


def _fp8_operands(specs):
    """MX e4m3 copies of 2-D operands (kdfm_fp8_quant_mx: one e8m0 scale per 32 consecutive contraction elements):
    specs = [(tensor f32 / bf16, transpose)], the transposed copy being the data gradient's W^T rows.  Returns
    [(address, row stride in bytes, scale-tensor address)]; the copies live in this stream's scratch."""
    dev = specs[0][0].device
    shapes = []
    for t, tr in specs:
        assert t.dim() == 2 and t.stride(1) == 1 and t.dtype in (torch.float32, torch.bfloat16)
        r, kc = (t.shape[1], t.shape[0]) if tr else (t.shape[0], t.shape[1])
        shapes.append((r, -(-kc // 16) * 16, kc))
    nbytes = sum(r * ld + -(-(r * kc // 32) // 16) * 16 for r, ld, kc in shapes)
    buf = scratch(dev, nbytes // 4 + 16)
    out, off = [], 0
    for (t, tr), (r, ld, kc) in zip(specs, shapes):
        dst = buf.data_ptr() + off
        off += r * ld
        sc = buf.data_ptr() + off
        off += -(-(r * kc // 32) // 16) * 16
        call("kdfm_fp8_quant_mx", ptr(t), 1 if t.dtype == torch.bfloat16 else 0, t.shape[0], t.shape[1], t.stride(0),
             dst, ld, sc, 1 if tr else 0, _s())
        out.append((dst, ld, sc))
    return out


def _big_out(out):
    """(f32 C tensor or None, bf16 C16 address or 0)."""
    if out.dtype == torch.bfloat16:
        assert out.stride(1) == 1
        return None, out.data_ptr()
    return _f32(out), 0


def _splitk_for(M, N, K):
    tiles = -(-M // 64) * -(-N // 64)
    if K <= 512 or tiles >= 256:
        return 1
    want = max(1, 512 // tiles)
    return int(min(want, max(1, K // 512), 1024))


def linear(x, W, bias, out, *, epi=0, R=None, rscale=1.0, Cpre=None, dropout_p=0.0, seed=None, rng_stream=0,
           alpha=1.0, math=None, rowmask=None, mse=None, tag=None):
    """out[M,N] = epi(alpha * x[M,K] @ W[N,K]^T + bias)   (W may be a strided view).  x / out may be bf16 on the
    large-tile route (big_ok(M, N, K, NT))."""
    M, K = x.shape
    N = W.shape[0]
    assert W.shape[1] == K and out.shape[0] == M and out.shape[1] == N, (x.shape, W.shape, out.shape)
    if bias is not None:
        epi |= _lib.EPI_BIAS
    if (math or _State.math) == "bf16" and mse is None and fp8_ok(M, N, K):
        wq = _fp8_weight(W, False)
        if wq is None:
            (a8, lda, sa), (w8, ldw, sw) = _fp8_operands([(x, False), (W, False)])
        else:
            ((a8, lda, sa),), (w8, ldw, sw) = _fp8_operands([(x, False)]), wq
        C, c16 = _big_out(out)
        side = sum(1 for t in (R, Cpre) if t is not None)
        nb = 1.0 * (M * K + N * K) + (2.0 if c16 else 4.0) * M * N + 4.0 * side * M * N
        gemm(x, W, C if C is not None else out, M, N, K, 0, 0, 0, 0, out.stride(0), out.stride(1), amode=_lib.LD_KC,
             bmode=_lib.LD_KC, epi=epi, bias=bias, R=R, rscale=rscale, Cpre=Cpre, dropout_p=dropout_p, seed=seed,
             rng_stream=rng_stream, alpha=alpha, rowmask=rowmask, tag=tag, nbytes=nb,
             fp8=(a8, lda, w8, ldw, sa, sw, c16))
        return
    if (math or _State.math) == "bf16" and mse is None and big_ok(M, N, K, _lib.BIG_NT):
        (a16, lda), (w16, ldw) = _bf16_operands((x, W), weight=1)
        C, c16 = _big_out(out)
        side = sum(1 for t in (R, Cpre) if t is not None)
        nb = 2.0 * (M * K + N * K) + (2.0 if c16 else 4.0) * M * N + 4.0 * side * M * N
        gemm(x, W, C if C is not None else out, M, N, K, 0, 0, 0, 0, out.stride(0), out.stride(1), amode=_lib.LD_KC,
             bmode=_lib.LD_KC, epi=epi, bias=bias, R=R, rscale=rscale, Cpre=Cpre, dropout_p=dropout_p, seed=seed,
             rng_stream=rng_stream, alpha=alpha, rowmask=rowmask, tag=tag, nbytes=nb,
             big=(a16, lda, w16, ldw, _lib.BIG_NT, c16))
        return
    _f32(x, "x")
    _f32(out, "out")
    gemm(x, W, out, M, N, K, x.stride(0), x.stride(1), W.stride(1), W.stride(0), out.stride(0), out.stride(1),
         amode=_lib.LD_KC, bmode=_lib.LD_KC, epi=epi, bias=bias, R=R, rscale=rscale, Cpre=Cpre,
         dropout_p=dropout_p, seed=seed, rng_stream=rng_stream, alpha=alpha, math=math, rowmask=rowmask, mse=mse,
         tag=tag, Bh=bf16_twin(W) if _TWINS else None)


def linear_dx(dy, W, dx, *, epi=0, aux=None, dropout_p=0.0, seed=None, rng_stream=0, R=None, rscale=1.0,
              alpha=1.0, math=None, rowmask=None):
    """dx[M,K] = epi(alpha * dy[M,N] @ W[N,K]).  dy / dx may be bf16 on the large-tile route (big_ok(M, K, N, NN))."""
    M, N = dy.shape
    K = W.shape[1]
    assert W.shape[0] == N and dx.shape[0] == M and dx.shape[1] == K, (dy.shape, W.shape, dx.shape)
    if R is not None:
        epi |= _lib.EPI_RESID
    if (math or _State.math) == "bf16" and fp8_ok(M, K, N):
        # dx = dY (W^T)^T: the fp8 instance is k-contiguous only, so W is quantised transposed ([K][N] rows)
        wq = _fp8_weight(W, True)
        if wq is None:
            (a8, lda, sa), (w8, ldw, sw) = _fp8_operands([(dy, False), (W, True)])
        else:
            ((a8, lda, sa),), (w8, ldw, sw) = _fp8_operands([(dy, False)]), wq
        C, c16 = _big_out(dx)
        side = sum(1 for t in (R, aux) if t is not None)
        nb = 1.0 * (M * N + N * K) + (2.0 if c16 else 4.0) * M * K + 4.0 * side * M * K
        gemm(dy, W, C if C is not None else dx, M, K, N, 0, 0, 0, 0, dx.stride(0), dx.stride(1), amode=_lib.LD_KC,
             bmode=_lib.LD_XC, epi=epi, aux=aux, dropout_p=dropout_p, seed=seed, rng_stream=rng_stream, R=R,
             rscale=rscale, alpha=alpha, rowmask=rowmask, nbytes=nb, fp8=(a8, lda, w8, ldw, sa, sw, c16))
        return
    if (math or _State.math) == "bf16" and big_ok(M, K, N, _lib.BIG_NN):
        (a16, lda), (w16, ldw) = _bf16_operands((dy, W), weight=1)
        C, c16 = _big_out(dx)
        side = sum(1 for t in (R, aux) if t is not None)
        nb = 2.0 * (M * N + N * K) + (2.0 if c16 else 4.0) * M * K + 4.0 * side * M * K
        gemm(dy, W, C if C is not None else dx, M, K, N, 0, 0, 0, 0, dx.stride(0), dx.stride(1), amode=_lib.LD_KC,
             bmode=_lib.LD_XC, epi=epi, aux=aux, dropout_p=dropout_p, seed=seed, rng_stream=rng_stream, R=R,
             rscale=rscale, alpha=alpha, rowmask=rowmask, nbytes=nb, big=(a16, lda, w16, ldw, _lib.BIG_NN, c16))
        return
    _f32(dy, "dy")
    _f32(dx, "dx")
    gemm(dy, W, dx, M, K, N, dy.stride(0), dy.stride(1), W.stride(0), W.stride(1), dx.stride(0), dx.stride(1),
         amode=_lib.LD_KC, bmode=_lib.LD_XC, epi=epi, aux=aux, dropout_p=dropout_p, seed=seed,
         rng_stream=rng_stream, R=R, rscale=rscale, alpha=alpha, math=math, rowmask=rowmask,
         Bh=bf16_twin(W, transposed=True) if _TWINS else None)


def linear_dw(dy, x, dW, *, alpha=1.0, math=None, db=None):
    """dW[N,K] += alpha * dy[M,N]^T @ x[M,K]; with db: db[N] += alpha * colsum(dy) fused as an
    implicit ones column of x (split-K, f32 atomics into the grad buffer)"""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dW.shape[0] == N and dW.shape[1] == K, (dy.shape, x.shape, dW.shape)
    if (math or _State.math) == "bf16" and big_ok(N, K, M, _lib.BIG_TN):
        # dW[n][k] += alpha sum_r dy[r][n] x[r][k]: both operands k-major (the rows are the reduction), one writer
        # per gradient element, the bias gradient from the same kernel (row sums of dy^T)
        (a16, lda), (b16, ldb) = _bf16_operands((dy, x))
        nb = 2.0 * M * (N + K) + 8.0 * N * K
        gemm(dy, x, dW, N, K, M, 0, 0, 0, 0, dW.stride(0), dW.stride(1), amode=_lib.LD_XC, bmode=_lib.LD_XC,
             epi=_lib.EPI_ATOMIC, alpha=alpha, ones_out=db, nbytes=nb, big=(a16, lda, b16, ldb, _lib.BIG_TN, 0))
        return
    _f32(dy, "dy")
    _f32(x, "x")
    Kx = K + (1 if db is not None else 0)
    sk = _splitk_for(N, Kx, M)
    gemm(dy, x, dW, N, Kx, M, dy.stride(1), dy.stride(0), x.stride(0), x.stride(1), dW.stride(0), dW.stride(1),
         amode=_lib.LD_XC, bmode=_lib.LD_XC, epi=_lib.EPI_ATOMIC, splitk=sk, alpha=alpha, math=math, ones_out=db)


def conv3(x, Wf, bias, out, T, *, epi=0, R=None, rscale=1.0, alpha=1.0, aux=None, math=None, tag=None):
    """Conv1d(k=3, pad=1) along frames on channels-last rows: out[r,o] = sum_{tap,c} Wf[o, tap*C+c] x[r+tap-1, c]
    Wf: (O, 3*C) GEMM layout from kdfm_convw_prep; rows grouped in utterances of T frames.
    Algorithmic bytes (bench roofline): x read once (the taps are re-reads of the same rows), the
    output and each side operand (R / aux) once, the weights once; all f32."""
    M, Cc = x.shape
    O = Wf.shape[0]
    assert Wf.shape[1] == 3 * Cc and x.stride(1) == 1
    if bias is not None:
        epi |= _lib.EPI_BIAS
    if R is not None:
        epi |= _lib.EPI_RESID
    gemm(x, Wf, out, M, O, 3 * Cc, x.stride(0), 1, 1, Wf.stride(0), out.stride(0), out.stride(1),
         amode=_lib.LD_CONV, bmode=_lib.LD_KC, epi=epi, bias=bias, R=R, rscale=rscale, alpha=alpha, aux=aux,
         conv=(3, 1, Cc, T), math=math, Bh=bf16_twin(Wf) if _TWINS else None, tag=tag,
         nbytes=4.0 * (M * Cc + M * O * (1 + (R is not None) + (aux is not None)) + O * 3 * Cc))


def conv3_dw(dy, x, G, T, *, alpha=1.0, math=None, db=None):
    """G[o, tap*C + c] += alpha * sum_r dy[r,o] x[r+tap-1, c]   (weight grad in GEMM layout);
    with db: db[o] += alpha * sum_r dy[r,o] (implicit ones column)"""
    M, O = dy.shape
    Cc = x.shape[1]
    assert G.shape == (O, 3 * Cc)
    Nx = 3 * Cc + (1 if db is not None else 0)
    sk = _splitk_for(O, Nx, M)
    gemm(dy, x, G, O, Nx, M, dy.stride(1), dy.stride(0), x.stride(0), 1, G.stride(0), 1,
         amode=_lib.LD_XC, bmode=_lib.LD_CONV, epi=_lib.EPI_ATOMIC, splitk=sk, alpha=alpha,
         conv=(3, 1, Cc, T), math=math, ones_out=db)


def colsum(x2d, out, *, scale=1.0, accumulate=True):
    M, N = x2d.shape
    assert x2d.stride(1) == 1 and out.numel() == N
    call("kdfm_colsum", ptr(x2d), ptr(out), M, N, x2d.stride(0), float(scale), int(accumulate), _s())


# ------------------------------------------------------------------------------------------------
# elementwise / glue
# ------------------------------------------------------------------------------------------------

def fill(x, value=0.0):
    assert x.is_contiguous()
    call("kdfm_fill", ptr(_f32(x)), float(value), x.numel(), _s())


def axpby(a, b, out, alpha=1.0, beta=1.0):
    """out = alpha*a + beta*b on 2-D (possibly row-strided) views; b may be None."""
    rows, cols = out.shape
    assert a.shape == out.shape and (b is None or b.shape == out.shape)
    assert a.stride(1) == 1 and out.stride(1) == 1 and (b is None or b.stride(1) == 1)
    call("kdfm_axpby", ptr(a), a.stride(0), ptr(b), b.stride(0) if b is not None else 0, ptr(out), out.stride(0),
         rows, cols, float(alpha), float(beta), _s())


def rowscale(x, out, s, rows_per_s, alpha=1.0):
    assert x.is_contiguous() and out.is_contiguous() and x.numel() == out.numel()
    rows = x.numel() // (x.shape[-1] if x.dim() > 1 else 1)
    cols = x.numel() // rows
    call("kdfm_rowscale", ptr(x), ptr(out), rows, cols, ptr(s), int(rows_per_s), float(alpha), _s())


def relu_mask(dy, y, out):
    assert dy.is_contiguous() and y.is_contiguous() and out.is_contiguous()
    call("kdfm_relu_mask", ptr(dy), ptr(y), ptr(out), y.numel(), _s())


def mse(a, b, loss_acc, scale, grad=None, gscale=0.0):
    assert a.is_contiguous() and b.is_contiguous() and a.numel() == b.numel()
    call("kdfm_mse", ptr(a), ptr(b), ptr(grad), ptr(loss_acc), a.numel(), float(scale), float(gscale), _s())


def l1(a, b, loss_acc, scale, grad=None, gscale=0.0):
    assert a.is_contiguous() and b.is_contiguous() and a.numel() == b.numel()
    call("kdfm_l1", ptr(a), ptr(b), ptr(grad), ptr(loss_acc), a.numel(), float(scale), float(gscale), _s())


def dropout(x, out, p, scale, seed, rng_stream):
    """out f32, or bf16 (rounded to nearest even: an operand only bf16-operand products read)."""
    assert x.is_contiguous() and out.is_contiguous() and x.numel() == out.numel()
    if out.dtype == torch.bfloat16:
        call("kdfm_dropout_bf16", ptr(x), out.data_ptr(), x.numel(), float(p), float(scale), ptr(seed),
             int(rng_stream), _s())
        return
    call("kdfm_dropout", ptr(x), ptr(out), x.numel(), float(p), float(scale), ptr(seed), int(rng_stream), _s())


def unfold1d(x, cols, B, Lin, Lrows, K=4, S=2, P=1, Lvalid=None):
    """cols[(b, i), k*C + c] = x[(b, S i - P + k), c] (0 outside [0, Lvalid), default Lin): x (B*Lin, C) rows, may be
    a column slice of a wider buffer (x.stride(1) == 1)."""
    C = x.shape[1]
    assert x.shape[0] == B * Lin and x.stride(1) == 1 and cols.shape == (B * Lrows, K * C) and cols.is_contiguous()
    call("kdfm_unfold1d", ptr(x), x.stride(0), ptr(cols), B, Lin, Lin if Lvalid is None else Lvalid, Lrows, C, K, S, P,
         _s())


def fold1d(cols, out, B, Lrows, Lout, *, K=4, S=2, P=1, bias=None, R=None, Lvalid=None):
    """out[(b, t), c] = R + [t < Lvalid] (bias + the taps of cols that land on t) (transposed-conv overlap-add;
    Lvalid defaults to Lout); out (B*Lout, C) may be a column slice of a wider buffer; R may alias out."""
    C = out.shape[1]
    assert out.shape[0] == B * Lout and out.stride(1) == 1 and cols.shape == (B * Lrows, K * C) and cols.is_contiguous()
    assert R is None or (R.shape == out.shape and R.stride(1) == 1)
    call("kdfm_fold1d", ptr(cols), ptr(out), out.stride(0), ptr(bias), ptr(R), R.stride(0) if R is not None else 0, B,
         Lrows, Lout, Lout if Lvalid is None else Lvalid, C, K, S, P, _s())


def convw_prep(W, fwd=None, bwd=None):
    O, I, K = W.shape
    call("kdfm_convw_prep", ptr(W.contiguous()), ptr(fwd), ptr(bwd), O, I, K, _s())


def convw_grad(G, dW, alpha=1.0):
    O, I, K = dW.shape
    assert G.numel() == dW.numel() and dW.is_contiguous()
    call("kdfm_convw_grad", ptr(G), ptr(dW), O, I, K, float(alpha), _s())


def subsample_lengths(wav_len, mel_len, len1, len2, hop):
    call("kdfm_subsample_lengths", ptr(_i64(wav_len)), ptr(mel_len), ptr(len1), ptr(len2), wav_len.numel(), hop, _s())


def step_advance(step, seed):
    call("kdfm_step_advance", ptr(step), ptr(seed), _s())


def relpos_table(T, d, out):
    assert out.shape == (2 * T - 1, d)
    call("kdfm_relpos_table", ptr(out), T, d, _s())


# ------------------------------------------------------------------------------------------------
# frontend / subsampling
# ------------------------------------------------------------------------------------------------

def preemph_pad(wav, lengths, xp, pad, preemph, dither, seed, rng_stream):
    B, N = wav.shape
    assert xp.shape == (B, N + 2 * pad) and wav.is_contiguous()
    call("kdfm_preemph_pad", ptr(_f32(wav)), ptr(_i64(lengths)), ptr(xp), B, N, pad, float(preemph),
         float(dither), ptr(seed), int(rng_stream), _s())


def logmel_fft(xp, window, twiddle, fb, fb_lo, fb_hi, mel, B, T, hop, n_fft, win):
    """mel (B*T, nfilt) = filterbank(|FFT_512(window * frame)|^2) per frame of the padded waveform xp."""
    nfilt = fb.shape[0]
    assert xp.shape[0] == B and xp.stride(1) == 1 and mel.shape == (B * T, nfilt) and fb.shape[1] == n_fft // 2 + 1
    assert twiddle.shape == (n_fft, 2) and fb_lo.dtype == torch.int32 and fb_hi.dtype == torch.int32
    call("kdfm_logmel_fft", ptr(_f32(xp)), xp.stride(0), ptr(_f32(window)), ptr(_f32(twiddle)), ptr(_f32(fb)),
         ptr(fb_lo), ptr(fb_hi), ptr(_f32(mel)), B, T, hop, n_fft, win, nfilt, _s())


def power_spectrum(spec, power):
    rows, F = power.shape
    assert spec.shape == (rows, 2 * F)
    call("kdfm_power_spectrum", ptr(spec), ptr(power), rows, F, _s())


def logmel_normalize(mel, seq_len, out, B, T, nf, guard):
    call("kdfm_logmel_normalize", ptr(mel), ptr(_i64(seq_len)), ptr(out), B, T, nf, float(guard), _s())


def specaugment(x, seq_len, B, T, nf, freq_masks, freq_width, time_masks, time_width, seed, rng_stream,
                mask_out=None, uniforms=None):
    """uniforms: optional (B, 2 (time_masks + freq_masks)) f32 draws in [0, 1) (parity mode: the RNG as an
    input), per utterance [time widths | time starts | freq widths | freq starts]; else the counter RNG."""
    if uniforms is not None:
        assert uniforms.dtype == torch.float32 and uniforms.is_contiguous()
        assert uniforms.numel() == B * 2 * (int(freq_masks) + int(time_masks))
    call("kdfm_specaugment", ptr(x), ptr(_i64(seq_len)), ptr(mask_out), B, T, nf, int(freq_masks),
         int(freq_width), int(time_masks), float(time_width), ptr(seed), int(rng_stream), ptr(uniforms), _s())


def im2col_3x3s2(X, len_in, cols, B, T1, F1, Cc):
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    assert cols.shape == (B * T2 * F2, 9 * Cc) and X.numel() == B * T1 * F1 * Cc
    call("kdfm_im2col_3x3s2", ptr(X), ptr(_i64(len_in)), ptr(cols), B, T1, F1, Cc, _s())


def im2col_3x3s2_tm_bf16(X, len_in, cols, B, T1, F1, Cc):
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    assert cols.shape == (B * T2 * F2, 9 * Cc) and cols.dtype == torch.bfloat16 and X.numel() == B * T1 * F1 * Cc
    if X.dtype == torch.bfloat16:
        call("kdfm_im2col_3x3s2_tm_from_bf16", ptr(X), ptr(_i64(len_in)), ptr(cols), B, T1, F1, Cc, _s())
        return
    call("kdfm_im2col_3x3s2_tm_bf16", ptr(_f32(X)), ptr(_i64(len_in)), ptr(cols), B, T1, F1, Cc, _s())


def col2im_3x3s2(dcols, len_in, relu_out, dX, B, T1, F1, Cc, tapmajor=False):
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    assert dcols.shape == (B * T2 * F2, 9 * Cc) and dX.numel() == B * T1 * F1 * Cc
    call("kdfm_col2im_3x3s2_tapmajor" if tapmajor else "kdfm_col2im_3x3s2", ptr(dcols), ptr(_i64(len_in)), ptr(relu_out), ptr(dX), B, T1, F1, Cc, _s())


def _bf16(t, name="tensor"):
    if t is not None and t.dtype != torch.bfloat16:
        raise _lib.KdfmError(f"{name} must be bfloat16, got {t.dtype}")
    return t


def wgrad_bf16_supported(rows, M, N, bias=True) -> bool:
    return int(_lib.lib().kdfm_wgrad_bf16_ws(int(rows), int(M), int(N), 1 if bias else 0)) >= 0


def wgrad_bf16(dY, X, dW, *, db=None, alpha=1.0):
    """dW[m, n] += alpha * dY[:, m]^T X[:, n] (+ db[m] += alpha * colsum(dY)), bf16 row operands,
    row-parallel MFMA kernel with an ordered fold.  dW may be a row-strided view (stride(1) == 1)."""
    rows, M = dY.shape
    N = X.shape[1]
    assert X.shape[0] == rows and dW.shape == (M, N) and dW.stride(1) == 1, (dY.shape, X.shape, dW.shape)
    assert dY.is_contiguous() and X.is_contiguous()
    n = int(_lib.lib().kdfm_wgrad_bf16_ws(rows, M, N, 1 if db is not None else 0))
    if n < 0:
        raise _lib.KdfmError(f"kdfm_wgrad_bf16: unsupported shape rows={rows} M={M} N={N}")
    ws = scratch(dY.device, n)
    # algorithmic bytes: both bf16 row operands once, the f32 gradient read + written
    _traced("wgrad_bf16", 2.0 * rows * M * N, 2.0 * rows * (M + N) + 8.0 * M * N, "kdfm_wgrad_bf16", ptr(_bf16(dY)),
            ptr(_bf16(X)), ptr(_f32(dW)), dW.stride(0), ptr(db), rows, M, N, float(alpha), ptr(ws), ws.numel(), _s())


def wgrad_set_fold_arena(arena):
    """Defer the ordered folds of the row-parallel weight gradients issued on the current stream: their
    partials go to `arena` (f32, None ends deferral) and wgrad_fold_flush() folds them in one launch."""
    assert arena is None or (arena.dtype == torch.float32 and arena.is_contiguous())
    call("kdfm_wgrad_set_fold_arena", _s(), ptr(arena), 0 if arena is None else arena.numel())


def wgrad_fold_flush():
    """Fold every weight gradient queued on the current stream (one launch per 24 products).  Traced as
    "wgrad_fold" (no algorithmic bytes of its own: the folds' time belongs to the deferred products')."""
    _traced("wgrad_fold", 0.0, 0.0, "kdfm_wgrad_fold_flush", _s())


def wgrad_fold_pending() -> int:
    return int(_lib.lib().kdfm_wgrad_fold_pending(_s()))


def wgrad_fold_stats(stream=None):
    """(queued folds, fallbacks since the arena was set, peak arena demand in floats) of `stream` (default: the
    current one): host-side bookkeeping of libkdfm, no device sync."""
    out = (C.c_int64 * 3)()
    sp = _s() if stream is None else stream
    _lib.check(_lib.lib().kdfm_wgrad_fold_stats(sp, out), "kdfm_wgrad_fold_stats")
    return int(out[0]), int(out[1]), int(out[2])


def wgrad_fold_discard_all() -> int:
    """Error recovery: drop every stream's queued deferred folds and unset every fold arena."""
    return int(_lib.lib().kdfm_wgrad_fold_discard_all())


def wgrad_bf16_pair(dY, X, dW, db, dY2, X2, dW2, db2, *, alpha=1.0):
    """Two same-shape weight gradients in one launch (kdfm_wgrad_bf16_pair): each equal bit for bit to its
    own wgrad_bf16; db / db2 both given or both None; dW and dW2 share the row stride."""
    rows, M = dY.shape
    N = X.shape[1]
    assert dY2.shape == dY.shape and X2.shape == X.shape and dW.shape == (M, N) and dW2.shape == (M, N)
    assert dW.stride(1) == 1 and dW2.stride(1) == 1 and dW.stride(0) == dW2.stride(0)
    assert (db is None) == (db2 is None)
    for t in (dY, X, dY2, X2):
        assert t.is_contiguous()
    n = int(_lib.lib().kdfm_wgrad_bf16_ws(rows, M, N, 1 if db is not None else 0))
    if n < 0:
        raise _lib.KdfmError(f"kdfm_wgrad_bf16_pair: unsupported shape rows={rows} M={M} N={N}")
    ws = scratch(dY.device, 2 * n)
    _traced("wgrad_bf16", 4.0 * rows * M * N, 2.0 * (2.0 * rows * (M + N) + 8.0 * M * N), "kdfm_wgrad_bf16_pair",
            ptr(_bf16(dY)), ptr(_bf16(X)), ptr(_f32(dW)), ptr(db), ptr(_bf16(dY2)), ptr(_bf16(X2)), ptr(_f32(dW2)),
            ptr(db2), dW.stride(0), rows, M, N, float(alpha), ptr(ws), ws.numel(), _s())


def wgrad_bf16_seg_ok(rows, M, N, seg_rows) -> bool:
    return int(_lib.lib().kdfm_wgrad_bf16_seg_ws(int(rows), int(M), int(N), int(seg_rows))) >= 0


def wgrad_bf16_seg(dY, X, dW, db, seg_rows, *, alpha=1.0):
    """dW[m, n] += alpha * dY[:, m]^T X[:, n] over all rows, and one bias gradient per stacked segment
    of seg_rows rows: db[j, m] += alpha * sum_{r in segment j} dY[r, m] (one launch + one fold)."""
    rows, M = dY.shape
    N = X.shape[1]
    nseg = rows // seg_rows
    assert X.shape[0] == rows and dW.shape == (M, N) and dW.stride(1) == 1, (dY.shape, X.shape, dW.shape)
    assert dY.is_contiguous() and X.is_contiguous() and db.shape == (nseg, M) and db.is_contiguous()
    n = int(_lib.lib().kdfm_wgrad_bf16_seg_ws(rows, M, N, seg_rows))
    if n < 0:
        raise _lib.KdfmError(f"kdfm_wgrad_bf16_seg: unsupported shape rows={rows} M={M} N={N} seg_rows={seg_rows}")
    ws = scratch(dY.device, n)
    _traced("wgrad_bf16", 2.0 * rows * M * N, 2.0 * rows * (M + N) + 8.0 * M * N, "kdfm_wgrad_bf16_seg",
            ptr(_bf16(dY)), ptr(_bf16(X)), ptr(_f32(dW)), dW.stride(0), ptr(_f32(db)), seg_rows, rows, M, N,
            float(alpha), ptr(ws), ws.numel(), _s())


def fm_chain_fwd(x0, zt, W1, cvec, W2, b2, Wst, bst, X, A, nsx, dtr, xS, loss, inv, S):
    n, L = x0.shape
    assert zt.shape == (n, L) and dtr.shape == (n, L) and W1.stride(1) == 1 and cvec.shape[0] >= S
    for t in (X, A):
        assert t is None or (t.shape == (S, n, L) and t.is_contiguous())
    call("kdfm_fm_chain_fwd", ptr(_f32(x0)), ptr(_f32(zt)), ptr(_f32(W1)), W1.stride(0), ptr(_f32(cvec)),
         ptr(_f32(W2)), ptr(_f32(b2)), ptr(_f32(Wst)), ptr(_f32(bst)), ptr(_bf16(X)), ptr(_bf16(A)), ptr(nsx),
         ptr(dtr), ptr(xS), ptr(loss), float(inv), n, L, S, _s())


def fm_chain_bwd(dtr, A, gxS, W1, W2, Wst, DV, DA, gx0, S):
    n, L = dtr.shape
    assert A.shape == (S, n, L) and gx0.shape == (n, L) and W1.stride(1) == 1
    for t in (DV, DA):
        assert t is None or (t.shape == (S, n, L) and t.is_contiguous())
    assert gxS is None or (gxS.shape == (n, L) and gxS.is_contiguous())
    call("kdfm_fm_chain_bwd", ptr(_f32(dtr)), ptr(_bf16(A)), ptr(_f32(gxS)), ptr(_f32(W1)), W1.stride(0),
         ptr(_f32(W2)), ptr(_f32(Wst)), ptr(_bf16(DV)), ptr(_bf16(DA)), ptr(gx0), n, L, S, _s())


def ffn_supported(d, ff) -> bool:
    return bool(_lib.lib().kdfm_ffn_supported(int(d), int(ff)))


def ffn_img(W1, W2, *, fwd_only=False, out=None):
    """bf16 chunk images of one feed-forward module's W1 (ff, d) / W2 (d, ff) for kdfm_ffn_fwd/bwd."""
    ff, d = W1.shape
    assert W2.shape == (d, ff) and W1.is_contiguous() and W2.is_contiguous()
    if _IMGSETS and out is None:
        img = _registered_img(IMG_FFN, 0, 0, W1)
        if img is None and fwd_only:
            img = _registered_img(IMG_FFN, 0, 1, W1)
        if img is not None:
            return img
    n = int(_lib.lib().kdfm_ffn_img_elems(d, ff))
    if n <= 0:
        raise _lib.KdfmError(f"kdfm_ffn: unsupported shape d={d} ff={ff}")
    img = out if out is not None else torch.empty(n, device=W1.device, dtype=torch.bfloat16)
    assert img.numel() >= n and img.dtype == torch.bfloat16
    call("kdfm_ffn_wprep", ptr(_f32(W1)), ptr(_f32(W2)), ptr(img), d, ff, int(bool(fwd_only)), _s())
    return img


def ffn_fwd(x, g, b, eps, img, b1, b2, out, mean, rstd, ff, *, rscale, p_act, p_out, seed, st_act, st_out,
            out_ln=None):
    """out = x + rscale * drop(W2 drop(silu(W1 LN(x) + b1)) + b2) (the fused macaron FFN block);
    out_ln = (gamma, beta, eps, y, mean, rstd): also y = LN(out) (the layer's norm_out) in the epilogue."""
    rows, d = x.shape
    assert out.shape == (rows, d) and x.is_contiguous() and out.is_contiguous()
    assert (mean is None) == (rstd is None)
    og, ob, oeps, oy, om, orr = out_ln if out_ln is not None else (None, None, 0.0, None, None, None)
    assert oy is None or (oy.shape == (rows, d) and oy.is_contiguous())
    # algorithmic bytes: x read, out written (+ the row statistics, + the LN output), weights once (bf16)
    nb = 8.0 * rows * d + 4.0 * d * ff + (8.0 * rows if mean is not None else 0.0) + \
        (4.0 * rows * d + 8.0 * rows if oy is not None else 0.0)
    _traced("ffn_fwd", 4.0 * rows * d * ff, nb, "kdfm_ffn_fwd", ptr(_f32(x)), ptr(_f32(g)), ptr(_f32(b)), float(eps),
            ptr(_bf16(img)), ptr(_f32(b1)), ptr(_f32(b2)), ptr(out), ptr(mean), ptr(rstd), rows, d, int(ff),
            float(rscale), float(p_act), float(p_out), ptr(seed), int(st_act), int(st_out), ptr(og), ptr(ob),
            float(oeps), ptr(oy), ptr(om), ptr(orr), _s())


def ffn_bwd(dout, x, mean, rstd, g, b, img, b1, dx, ln_h, a_h, dl2_h, dh_h, part, ff, *, rscale, p_act, p_out, seed,
            st_act, st_out):
    rows, d = x.shape
    assert dout.shape == (rows, d) and dx.shape == (rows, d) and dout.is_contiguous() and dx.is_contiguous()
    assert ln_h.shape == (rows, d) and dl2_h.shape == (rows, d) and a_h.shape == (rows, ff) and dh_h.shape == (rows, ff)
    assert part.numel() >= layernorm_bwd_ws(rows, d)
    # algorithmic bytes: dout, x read; dx written (f32); ln, dl2 (bf16, d wide), a, dh (bf16, ff wide)
    # written; row statistics read; weights once
    nb = 12.0 * rows * d + 8.0 * rows + 4.0 * rows * d + 4.0 * rows * ff + 4.0 * d * ff
    _traced("ffn_bwd", 6.0 * rows * d * ff, nb, "kdfm_ffn_bwd", ptr(_f32(dout)), ptr(_f32(x)), ptr(_f32(mean)),
            ptr(_f32(rstd)), ptr(_f32(g)), ptr(_f32(b)), ptr(_bf16(img)), ptr(_f32(b1)), ptr(dx), ptr(_bf16(ln_h)),
            ptr(_bf16(a_h)), ptr(_bf16(dl2_h)), ptr(_bf16(dh_h)), ptr(part), rows, d, int(ff), float(rscale),
            float(p_act), float(p_out), ptr(seed), int(st_act), int(st_out), _s())


RG_PRO_NONE, RG_PRO_DROP, RG_PRO_BNSILU = 0, 1, 2
RG_EPI_NONE, RG_EPI_RESID = 0, 1


def rowgemm_supported(d) -> bool:
    return int(_lib.lib().kdfm_rowgemm_img_elems(int(d))) > 0


def rowgemm_img(W, *, trans=False):
    """bf16 fragment image of a (d, d) weight for kdfm_rowgemm (trans: the data-gradient product)."""
    d = W.shape[0]
    assert W.shape == (d, d) and W.is_contiguous()
    if _IMGSETS:
        img = _registered_img(IMG_ROWGEMM, 0, int(bool(trans)), W)
        if img is not None:
            return img
    n = int(_lib.lib().kdfm_rowgemm_img_elems(d))
    if n <= 0:
        raise _lib.KdfmError(f"kdfm_rowgemm: unsupported d={d}")
    img = torch.empty(n, device=W.device, dtype=torch.bfloat16)
    call("kdfm_rowgemm_wprep", ptr(_f32(W)), ptr(img), d, int(bool(trans)), _s())
    return img


def rowgemm(x, img, out, *, pro=0, p_in=0.0, s_in=1.0, st_in=0, bn=None, x_h=None, epi=0, bias=None, R=None,
            rscale=1.0, p_out=0.0, st_out=0, seed=None):
    """out = epi(pro(x) Wop^T) over d-wide rows (kdfm_rowgemm); bn = (mean, rstd, gamma, beta)."""
    rows, d = x.shape
    assert out.shape == (rows, d) and x.is_contiguous() and out.is_contiguous()
    bm, br, bg, bb = bn if bn is not None else (None, None, None, None)
    call("kdfm_rowgemm", ptr(_f32(x)), ptr(_bf16(img)), ptr(out), rows, d, int(pro), float(p_in), float(s_in),
         int(st_in), ptr(bm), ptr(br), ptr(bg), ptr(bb), ptr(_bf16(x_h)), int(epi), ptr(_f32(bias)), ptr(_f32(R)),
         float(rscale), float(p_out), int(st_out), ptr(seed), _s())


LNPROJ_QKV, LNPROJ_GLU = 0, 1
IMG_FFN, IMG_LNPROJ, IMG_ROWGEMM = 0, 1, 2


_IMGSETS: list = []


def _registered_img(typ, kind, flag, W):
    p = W.data_ptr()
    for r in _IMGSETS:
        ws = r()
        if ws is not None:
            img = ws.by_weight.get((typ, kind, flag, p))
            if img is not None:
                return img
    return None


class WeightImages:
    """Every fused-kernel weight image of one model in ONE bf16 buffer, rebuilt by ONE launch
    (kdfm_wimg_prep_batch) whenever the f32 weights change (the engine: at the top of each step).
    Jobs are registered with add(); finalize() sizes the buffer and uploads the job table."""
    _FMT = struct.Struct("@5q3Pq")   # kdfm_wimg_job: type, kind, flag, d, ff, W1, W2, img, start

    def __init__(self, device):
        self.device = device
        self.specs = []    # (key, type, kind, flag, d, ff, W1, W2)
        self.imgs = {}
        self.table = None

    def add(self, key, typ, W1, W2=None, *, kind=0, flag=0, d=0, ff=0):
        assert self.table is None and W1.is_contiguous() and (W2 is None or W2.is_contiguous())
        self.specs.append((key, typ, kind, int(flag), int(d), int(ff), W1, W2))

    def _elems(self, typ, kind, flag, d, ff):
        lib = _lib.lib()
        if typ == IMG_FFN:
            return int(lib.kdfm_ffn_img_elems(d, ff))
        if typ == IMG_LNPROJ:
            return int(lib.kdfm_lnproj_img_elems(kind, d, flag))
        return int(lib.kdfm_rowgemm_img_elems(d))

    def finalize(self):
        sizes = [self._elems(t, k, f, d, ff) for _, t, k, f, d, ff, _, _ in self.specs]
        total = sum(sizes)
        if total == 0:
            return self
        self.buf = torch.empty(total, device=self.device, dtype=torch.bfloat16)
        raw = bytearray()
        off = start = 0
        one = C.create_string_buffer(self._FMT.size)
        for (key, t, k, f, d, ff, W1, W2), n in zip(self.specs, sizes):
            img = self.buf[off:off + n]
            self._FMT.pack_into(one, 0, t, k, f, d, ff, W1.data_ptr(), W2.data_ptr() if W2 is not None else 0,
                                img.data_ptr(), start)
            nthr = int(_lib.lib().kdfm_wimg_job_threads(one))
            if nthr <= 0:
                raise _lib.KdfmError(f"kdfm_wimg_job_threads: unsupported image {key}")
            raw += one.raw
            self.imgs[key] = img
            off += n
            start += nthr
        self.total_threads = start
        self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self.keep = [s[6:] for s in self.specs]   # the weight views stay alive with the table
        return self

    def register(self):
        """Make ffn_img / lnproj_img / rowgemm_img return these images for their weights."""
        import weakref
        _IMGSETS[:] = [r for r in _IMGSETS if r() is not None and r() is not self]
        _IMGSETS.append(weakref.ref(self))
        self.by_weight = {(t, k, f, W1.data_ptr()): self.imgs[key] for key, t, k, f, d, ff, W1, W2 in self.specs}
        return self

    def refresh(self):
        if self.table is not None:
            call("kdfm_wimg_prep_batch", ptr(self.table), len(self.imgs), self.total_threads, _s())

    def get(self, key):
        return self.imgs.get(key)


def lnproj_supported(kind, d, bwd=False) -> bool:
    return int(_lib.lib().kdfm_lnproj_img_elems(int(kind), int(d), int(bool(bwd)))) > 0


def lnproj_img(kind, W, *, bwd=False):
    """bf16 fragment image of a LayerNorm-fused projection weight W ((3d | 2d), d) fp32."""
    d = W.shape[1]
    assert W.is_contiguous() and W.shape[0] == (3 if kind == LNPROJ_QKV else 2) * d
    if _IMGSETS:
        img = _registered_img(IMG_LNPROJ, int(kind), int(bool(bwd)), W)
        if img is not None:
            return img
    n = int(_lib.lib().kdfm_lnproj_img_elems(int(kind), d, int(bool(bwd))))
    if n <= 0:
        raise _lib.KdfmError(f"kdfm_lnproj: unsupported kind={kind} d={d} bwd={bwd}")
    img = torch.empty(n, device=W.device, dtype=torch.bfloat16)
    call("kdfm_lnproj_wprep", int(kind), ptr(_f32(W)), ptr(img), d, int(bool(bwd)), _s())
    return img


def ln_qkv_fwd(x, g, b, eps, img, bias, pos_u, pos_v, qu, qv, qkv, mean=None, rstd=None, ln_h=None):
    rows, d = x.shape
    assert qu.shape == (rows, d) and qv.shape == (rows, d) and qkv.shape == (rows, 3 * d) and x.is_contiguous()
    call("kdfm_ln_qkv_fwd", ptr(_f32(x)), ptr(_f32(g)), ptr(_f32(b)), float(eps), ptr(_bf16(img)), ptr(_f32(bias)),
         ptr(_f32(pos_u)), ptr(_f32(pos_v)), ptr(qu), ptr(qv), ptr(qkv), ptr(mean), ptr(rstd), ptr(_bf16(ln_h)), rows, d,
         _s())


def ln_glu_fwd(x, g, b, eps, img, bias, lengths, T, gout, mean=None, rstd=None, ln_h=None):
    rows, d = x.shape
    assert gout.shape == (rows, d) and x.is_contiguous() and rows % T == 0
    call("kdfm_ln_glu_fwd", ptr(_f32(x)), ptr(_f32(g)), ptr(_f32(b)), float(eps), ptr(_bf16(img)), ptr(_f32(bias)),
         ptr(_i64(lengths)), int(T), ptr(gout), ptr(mean), ptr(rstd), ptr(_bf16(ln_h)), rows, d, _s())


def ln_qkv_bwd(dqu, dqv, dqkv, x, mean, rstd, g, b, img, dres, dx, ln_h, dqkv_h, part, part_uv=None):
    rows, d = x.shape
    assert dqkv.shape == (rows, 3 * d) and dqkv_h.shape == (rows, 3 * d) and ln_h.shape == (rows, d)
    assert part.numel() >= layernorm_bwd_ws(rows, d)
    assert part_uv is None or part_uv.numel() >= layernorm_bwd_ws(rows, d)
    call("kdfm_ln_qkv_bwd", ptr(_f32(dqu)), ptr(_f32(dqv)), ptr(_f32(dqkv)), ptr(_f32(x)), ptr(_f32(mean)),
         ptr(_f32(rstd)), ptr(_f32(g)), ptr(_f32(b)), ptr(_bf16(img)), ptr(_f32(dres)), ptr(dx), ptr(_bf16(ln_h)),
         ptr(_bf16(dqkv_h)), ptr(part), ptr(part_uv), rows, d, _s())


def ln_glu_bwd(dg, x, mean, rstd, g, b, img, bias, lengths, T, dres, dx, ln_h, da_h, part):
    rows, d = x.shape
    assert dg.shape == (rows, d) and da_h.shape == (rows, 2 * d) and ln_h.shape == (rows, d)
    assert part.numel() >= layernorm_bwd_ws(rows, d)
    call("kdfm_ln_glu_bwd", ptr(_f32(dg)), ptr(_f32(x)), ptr(_f32(mean)), ptr(_f32(rstd)), ptr(_f32(g)), ptr(_f32(b)),
         ptr(_bf16(img)), ptr(_f32(bias)), ptr(_i64(lengths)), int(T), ptr(_f32(dres)), ptr(dx), ptr(_bf16(ln_h)),
         ptr(_bf16(da_h)), ptr(part), rows, d, _s())


def wgrad_bf16_conv(dY, X, dW, T, *, taps=3, pad=1, db=None, alpha=1.0):
    """Conv1d weight gradient over utterances of T frames, bf16 row operands:
    dW[m, tap*C + c] += alpha * sum_r dY[r, m] X[r + tap - pad, c] (GEMM layout of convw_prep)."""
    rows, M = dY.shape
    C = X.shape[1]
    assert X.shape[0] == rows and dW.shape == (M, taps * C) and dW.stride(1) == 1 and rows % T == 0
    assert dY.is_contiguous() and X.is_contiguous()
    n = int(_lib.lib().kdfm_wgrad_bf16_conv_ws(rows, M, C, taps, pad, T, 1 if db is not None else 0))
    if n < 0:
        raise _lib.KdfmError(f"kdfm_wgrad_bf16_conv: unsupported shape rows={rows} M={M} C={C}")
    ws = scratch(dY.device, n)
    call("kdfm_wgrad_bf16_conv", ptr(_bf16(dY)), ptr(_bf16(X)), ptr(_f32(dW)), dW.stride(0), ptr(db), rows, M, C,
         taps, pad, T, float(alpha), ptr(ws), ws.numel(), _s())


def _img_ld(X, npos, C, what):
    """Row stride of a channels-last image of npos positions whose rows may be padded past C channels
    (kdfm_subsample_fused writes y1 rows of 32 ceil(C / 32) channels)."""
    ld = X.numel() // max(npos, 1)
    if ld * npos != X.numel() or ld < C or ld % 8 and ld != C:
        raise _lib.KdfmError(f"{what}: {X.numel()} elements are not {npos} rows of >= {C} channels")
    return ld


def wgrad_bf16_s2conv(dY, X, len_in, dW, db, B, T1, F1, C, *, alpha=1.0):
    """Striding subsampling conv2 weight gradient straight from its bf16 input X (B, T1, F1, ldx >= C) (no column
    matrix): dW (C, 9C) tap-major += alpha * sum dY[(b,t2,f2), m] X[b, 2t2-1+tap//3, 2f2-1+tap%3, c], db += colsum."""
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    rows = B * T2 * F2
    ldx = _img_ld(X, B * T1 * F1, C, "wgrad_bf16_s2conv X")
    assert dY.shape == (rows, C) and dW.shape == (C, 9 * C) and dW.is_contiguous()
    assert dY.is_contiguous() and X.is_contiguous() and db is not None
    n = int(_lib.lib().kdfm_wgrad_bf16_s2conv_ws(B, T1, F1, C))
    if n < 0:
        raise _lib.KdfmError(f"kdfm_wgrad_bf16_s2conv: unsupported shape B={B} T1={T1} F1={F1} C={C}")
    ws = scratch(dY.device, n)
    # algorithmic bytes: dY and X once (bf16), the f32 gradient read + written
    _traced("wgrad_bf16", 2.0 * rows * C * 9 * C, 2.0 * (rows * C + B * T1 * F1 * C) + 8.0 * 9 * C * C,
            "kdfm_wgrad_bf16_s2conv", ptr(_bf16(dY)), ptr(_bf16(X)), ldx, ptr(_i64(len_in)), ptr(_f32(dW)), ptr(_f32(db)),
            B, T1, F1, C, float(alpha), ptr(ws), ws.numel(), _s())


def denoise_chain_fwd(z, W1, b1, W2, b2, X, A, out, T, S):
    """Fused SimpleDenoiser forward (S steps) over utterances of T frames; W1/W2 Conv1d (L, L, 3)."""
    n, L = z.shape
    assert out.shape == (n, L) and n % T == 0 and W1.shape == (L, L, 3) and W2.shape == (L, L, 3)
    for t in (X, A):
        assert t is None or (t.shape == (S, n, L) and t.is_contiguous())
    wimg = torch.empty(int(_lib.lib().kdfm_denoise_wimg_elems()), device=z.device, dtype=torch.bfloat16)
    call("kdfm_denoise_chain_fwd", ptr(_f32(z)), ptr(_f32(W1.contiguous())), ptr(_f32(b1)), ptr(_f32(W2.contiguous())),
         ptr(_f32(b2)), ptr(wimg), ptr(_bf16(X)), ptr(_bf16(A)), ptr(_f32(out)), n, T, L, S, _s())


def denoise_chain_bwd(gout, A, W1, W2, GV, DA, gin, T, S):
    """Fused SimpleDenoiser data-gradient backward: gin = dL/dx_0 from gout = dL/dx_S; saves GV, DA."""
    n, L = gout.shape
    assert A.shape == (S, n, L) and gin.shape == (n, L) and n % T == 0
    for t in (GV, DA):
        assert t is None or (t.shape == (S, n, L) and t.is_contiguous())
    wimg = torch.empty(int(_lib.lib().kdfm_denoise_wimg_elems()), device=gout.device, dtype=torch.bfloat16)
    call("kdfm_denoise_chain_bwd", ptr(_f32(gout)), ptr(_bf16(A)), ptr(_f32(W1.contiguous())),
         ptr(_f32(W2.contiguous())), ptr(wimg), ptr(_bf16(GV)), ptr(_bf16(DA)), ptr(_f32(gin)), n, T, L, S, _s())


def conv_lengths(inp, out, pad_total, kernel=3, stride=2):
    """NeMo calc_length for one conv stage: out = floor((in + pad_total - kernel) / stride) + 1."""
    assert out.numel() == inp.numel() and out.dtype == torch.int64
    call("kdfm_conv_lengths", ptr(_i64(inp)), ptr(out), inp.numel(), int(pad_total), int(kernel), int(stride), _s())


def _dws_sizes(B, Ti, Fi, C, To, Fo):
    assert C % 4 == 0, "dw_striding channels must be a multiple of 4"
    return B * Ti * Fi * C, B * To * Fo * C


def dwsub_conv(x, in_len, w, b, y, out_len, B, Ti, Fi, Cin, C, To, Fo, pad, relu):
    """3x3 stride-2 conv of dw_striding subsampling (Cin 1: first stage; Cin C: depthwise)."""
    nin, nout = _dws_sizes(B, Ti, Fi, C, To, Fo)
    assert x.numel() == nin // C * Cin and y.numel() == nout and w.numel() == 9 * C and b.numel() == C
    assert x.is_contiguous() and y.is_contiguous()
    call("kdfm_dwsub_conv", ptr(_f32(x)), ptr(_i64(in_len)), ptr(_f32(w)), ptr(_f32(b)), ptr(y), ptr(_i64(out_len)),
         B, Ti, Fi, Cin, C, To, Fo, int(pad), int(pad), int(bool(relu)), _s())


def dwsub_conv_dgrad(dy, out_len, w, x_saved, in_len, dx, B, Ti, Fi, C, To, Fo, pad):
    nin, nout = _dws_sizes(B, Ti, Fi, C, To, Fo)
    assert dy.numel() == nout and dx.numel() == nin and (x_saved is None or x_saved.numel() == nin)
    call("kdfm_dwsub_conv_dgrad", ptr(_f32(dy)), ptr(_i64(out_len)), ptr(_f32(w)), ptr(x_saved), ptr(_i64(in_len)),
         ptr(dx), B, Ti, Fi, C, To, Fo, int(pad), int(pad), _s())


def dwsub_conv_wgrad(dy, out_len, x, in_len, dw, db, B, Ti, Fi, Cin, C, To, Fo, pad, accumulate=True):
    nin, nout = _dws_sizes(B, Ti, Fi, C, To, Fo)
    assert dy.numel() == nout and x.numel() == nin // C * Cin and dw.numel() == 9 * C and db.numel() == C
    n = int(_lib.lib().kdfm_dwsub_conv_wgrad_ws(B, To, Fo, C))
    ws = scratch(dy.device, n)
    call("kdfm_dwsub_conv_wgrad", ptr(_f32(dy)), ptr(_i64(out_len)), ptr(_f32(x)), ptr(_i64(in_len)), ptr(dw), ptr(db),
         ptr(ws), ws.numel(), B, Ti, Fi, Cin, C, To, Fo, int(pad), int(pad), int(bool(accumulate)), _s())


def subsample_wprep(w2, wb):
    """conv2 weight (C, C, 3, 3) f32 -> the bf16 [Np][9][Cp] image kdfm_subsample_conv2 reads"""
    Cc = w2.shape[0]
    assert w2.numel() == Cc * Cc * 9 and wb.dtype == torch.bfloat16
    assert wb.numel() >= _lib.lib().kdfm_subsample_wprep_elems(Cc)
    call("kdfm_subsample_wprep", ptr(_f32(w2)), ptr(wb), Cc, _s())


def subsample_wprep_elems(Cc):
    return int(_lib.lib().kdfm_subsample_wprep_elems(Cc))


def subsample_conv1(mel, mel_len, len1, w0, b0, y1b, y1f, B, Tm, F, Cc):
    T1, F1 = (Tm - 1) // 2 + 1, (F - 1) // 2 + 1
    assert mel.numel() == B * Tm * F and mel.is_contiguous()
    assert y1b.dtype == torch.bfloat16 and y1b.numel() == B * T1 * F1 * Cc
    assert y1f is None or y1f.numel() == B * T1 * F1 * Cc
    assert w0.numel() == Cc * 9 and b0.numel() == Cc
    call("kdfm_subsample_conv1", ptr(_f32(mel)), ptr(_i64(mel_len)), ptr(_i64(len1)), ptr(_f32(w0)), ptr(_f32(b0)),
         ptr(y1b), ptr(y1f), B, Tm, F, Cc, _s())


def subsample_conv2(y1b, len2, wb, b2, y2, B, T1, F1, Cc):
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    assert y1b.dtype == torch.bfloat16 and y1b.numel() == B * T1 * F1 * Cc
    assert y2.numel() == B * T2 * F2 * Cc and wb.dtype == torch.bfloat16
    call("kdfm_subsample_conv2", ptr(y1b), ptr(_i64(len2)), ptr(wb), ptr(_f32(b2)), ptr(_f32(y2)), B, T1, F1, Cc, _s())


def subsample_fused_supported(Cc, F=80):
    return bool(_lib.lib().kdfm_subsample_fused_supported(int(Cc), int(F)))


def subsample_fused_wprep_elems(Cc):
    return int(_lib.lib().kdfm_subsample_fused_wprep_elems(Cc))


def subsample_fused_wprep(w0, w2, wp):
    """conv1 (C, 1, 3, 3) and conv2 (C, C, 3, 3) f32 weights -> the bf16 operand image of
    kdfm_subsample_fused (conv1 as hi/lo bf16 splits, conv2 as [tap][chunk][co][32 ci] slabs)."""
    Cc = w2.shape[0]
    assert w0.numel() == Cc * 9 and w2.numel() == Cc * Cc * 9 and wp.dtype == torch.bfloat16
    assert wp.numel() >= subsample_fused_wprep_elems(Cc)
    call("kdfm_subsample_fused_wprep", ptr(_f32(w0)), ptr(_f32(w2)), ptr(wp), Cc, _s())


def subsample_fused(mel, mel_len, len1, len2, wp, b0, b2, y2, y1, B, Tm, F, Cc):
    """Striding subsampling forward in one kernel: y2 (B*T2*F2, C) f32; y1 (optional, (B*T1*F1, ldy1) bf16, ldy1 in
    [C, 32 ceil(C / 32)], the padding channels written as zeros) receives the conv1 output (kdfm_subsample_fused)."""
    T1, F1 = (Tm - 1) // 2 + 1, (F - 1) // 2 + 1
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    assert mel.numel() == B * Tm * F and mel.is_contiguous() and wp.dtype == torch.bfloat16
    assert y2.numel() == B * T2 * F2 * Cc and y2.is_contiguous()
    assert y1 is None or (y1.dtype == torch.bfloat16 and y1.is_contiguous())
    ldy1 = Cc if y1 is None else _img_ld(y1, B * T1 * F1, Cc, "subsample_fused y1")
    assert b0.numel() == Cc and b2.numel() == Cc
    call("kdfm_subsample_fused", ptr(_f32(mel)), ptr(_i64(mel_len)), ptr(_i64(len1)), ptr(_i64(len2)), ptr(wp),
         ptr(_f32(b0)), ptr(_f32(b2)), ptr(_f32(y2)), ptr(y1), B, Tm, F, Cc, ldy1, _s())


def subsample_dgrad_wprep_elems(Cc):
    return int(_lib.lib().kdfm_subsample_dgrad_wprep_elems(Cc))


def subsample_conv2_dgrad_w0(dy2, wt, y1, B, T1, F1, Cc, mel, mel_len, Tm, Fm, pad, dw0, db0, dy1=None):
    """conv2 data gradient (as subsample_conv2_dgrad) with conv0's weight gradient fused into the epilogue:
    dw0 (C, 9) += sum dy1 x_patch(mel), db0 (C) += sum dy1; dy1 optional."""
    assert dw0.numel() == Cc * 9 and dw0.is_contiguous() and db0.numel() == Cc
    n = int(_lib.lib().kdfm_subsample_conv2_dgrad_w0_ws(B, T1, F1, Cc))
    ws = scratch(dy2.device, n)
    ldy1 = _img_ld(y1, B * T1 * F1, Cc, "subsample_conv2_dgrad_w0 y1")
    call("kdfm_subsample_conv2_dgrad_w0", ptr(_f32(dy2)), ptr(wt), ptr(_bf16(y1, "y1 (bf16 conv1 output)")), ptr(dy1),
         B, T1, F1, Cc, ldy1, ptr(_f32(mel)), ptr(_i64(mel_len)), Tm, Fm, pad, ptr(_f32(dw0)), ptr(_f32(db0)), ptr(ws),
         ws.numel(), _s())


def subsample_conv2_dgrad_w0_h(dy2h, wt, y1, B, T1, F1, Cc, mel, mel_len, Tm, Fm, pad, dw0, db0, dy1=None):
    """subsample_conv2_dgrad_w0 over a bf16 dy2 (ss_out_dgrad's output)."""
    assert dw0.numel() == Cc * 9 and dw0.is_contiguous() and db0.numel() == Cc
    n = int(_lib.lib().kdfm_subsample_conv2_dgrad_w0_ws(B, T1, F1, Cc))
    ws = scratch(dy2h.device, n)
    ldy1 = _img_ld(y1, B * T1 * F1, Cc, "subsample_conv2_dgrad_w0_h y1")
    call("kdfm_subsample_conv2_dgrad_w0_h", ptr(_bf16(dy2h, "dy2h")), ptr(wt), ptr(_bf16(y1, "y1 (bf16 conv1 output)")),
         ptr(dy1), B, T1, F1, Cc, ldy1, ptr(_f32(mel)), ptr(_i64(mel_len)), Tm, Fm, pad, ptr(_f32(dw0)), ptr(_f32(db0)),
         ptr(ws), ws.numel(), _s())


def ss_out_wprep_elems(d, ncols):
    return int(_lib.lib().kdfm_ss_out_wprep_elems(d, ncols))


def ss_out_wprep(W, wt):
    """wt = bf16 W^T [ncols][32 ceil(d/32)] of the subsampling output weight W (d, ncols) (kdfm_ss_out_wprep)."""
    d, ncols = W.shape
    assert wt.dtype == torch.bfloat16 and wt.numel() >= int(_lib.lib().kdfm_ss_out_wprep_elems(d, ncols))
    call("kdfm_ss_out_wprep", ptr(_f32(W.contiguous())), ptr(wt), d, ncols, _s())


def ss_out_dgrad(dlin, wt, y2, dy2h):
    """dy2h (rows, ncols) bf16 = [y2 > 0] * (dlin @ W) with wt from ss_out_wprep (kdfm_ss_out_dgrad)."""
    rows, d = dlin.shape
    ncols = y2.shape[1]
    assert dlin.is_contiguous() and y2.shape[0] == rows and y2.is_contiguous() and dy2h.shape == (rows, ncols)
    call("kdfm_ss_out_dgrad", ptr(_f32(dlin)), ptr(wt), ptr(_f32(y2)), ptr(_bf16(dy2h, "dy2h")), rows, d, ncols, _s())


def subsample_dgrad_supported(Cc):
    """Channel counts the direct conv2 data-gradient kernel is instantiated for."""
    return Cc % 8 == 0 and ((-(-Cc // 32), -(-Cc // 16)) in ((3, 6), (1, 1), (1, 2), (2, 4)))


def subsample_dgrad_wprep(w2, wt):
    Cc = w2.shape[0]
    assert wt.dtype == torch.bfloat16 and wt.numel() >= subsample_dgrad_wprep_elems(Cc)
    call("kdfm_subsample_dgrad_wprep", ptr(_f32(w2.contiguous())), ptr(wt), Cc, _s())


def subsample_conv2_dgrad(dy2, wt, y1, dy1, B, T1, F1, Cc):
    """dy1 = [y1 > 0] * conv2^T(dy2) (stride-2 3x3 transposed conv, no im2col); dy2 (B T2 F2, C),
    y1 / dy1 (B T1 F1, C) channels-last f32."""
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    ldy1 = _img_ld(y1, B * T1 * F1, Cc, "subsample_conv2_dgrad y1")
    assert dy2.numel() == B * T2 * F2 * Cc and dy1.numel() == B * T1 * F1 * Cc
    call("kdfm_subsample_conv2_dgrad", ptr(_f32(dy2)), ptr(wt), ptr(_bf16(y1, "y1 (bf16 conv1 output)")), ptr(_f32(dy1)),
         B, T1, F1, Cc, ldy1, _s())


# ------------------------------------------------------------------------------------------------
# conformer layer pieces
# ------------------------------------------------------------------------------------------------

def layernorm_fwd(x, g, b, y, mean, rstd, eps):
    """y f32, or bf16 (d % 256 == 0: layernorm_bf16_ok) for an output only bf16-operand products read."""
    rows, d = x.shape
    assert x.is_contiguous() and y.is_contiguous() and mean.numel() == rows
    if y.dtype == torch.bfloat16:
        assert layernorm_bf16_ok(d)
        call("kdfm_layernorm_fwd_bf16", ptr(x), ptr(g), ptr(b), y.data_ptr(), ptr(mean), ptr(rstd), rows, d,
             float(eps), _s())
        return
    call("kdfm_layernorm_fwd", ptr(x), ptr(g), ptr(b), ptr(y), ptr(mean), ptr(rstd), rows, d, float(eps), _s())


def layernorm_bf16_ok(d) -> bool:
    """kdfm_layernorm_fwd_bf16 takes this width (the 16-byte-lane kernel: d % 256 == 0, d <= 1024)."""
    return d % 256 == 0 and d <= 1024


def layernorm_bwd(dy, x, g, mean, rstd, dx, dg, db, dres=None):
    rows, d = x.shape
    assert dy.is_contiguous() and dx.is_contiguous() and (dres is None or dres.is_contiguous())
    ws = scratch(x.device, _lib.lib().kdfm_layernorm_bwd_ws(rows, d))
    call("kdfm_layernorm_bwd", ptr(dy), ptr(x), ptr(g), ptr(mean), ptr(rstd), ptr(dres), ptr(dx), ptr(dg), ptr(db),
         ptr(ws), rows, d, _s())


def layernorm_bwd_ws(rows, d):
    return int(_lib.lib().kdfm_layernorm_bwd_ws(rows, d))


def layernorm_bwd_part(dy, x, g, mean, rstd, dx, part, dres=None, dy2=None):
    """LayerNorm backward with the dgamma/dbeta fold deferred to ln_fold (part: >= layernorm_bwd_ws
    floats, kept until the fold); dy2: a second output gradient summed into dy on load."""
    rows, d = x.shape
    assert dy.is_contiguous() and dx.is_contiguous() and (dres is None or dres.is_contiguous())
    assert part.numel() >= layernorm_bwd_ws(rows, d)
    if dy2 is not None:
        assert dy2.is_contiguous() and dy2.shape == dy.shape
        call("kdfm_layernorm_bwd_part2", ptr(dy), ptr(dy2), ptr(x), ptr(g), ptr(mean), ptr(rstd), ptr(dres), ptr(dx),
             ptr(part), rows, d, _s())
        return
    call("kdfm_layernorm_bwd_part", ptr(dy), ptr(x), ptr(g), ptr(mean), ptr(rstd), ptr(dres), ptr(dx), ptr(part),
         rows, d, _s())


def ln_fold(entries, rows, d):
    """entries: [(part, dgamma, dbeta)] (<= 8) of LayerNorms over the same (rows, d): one launch."""
    n = len(entries)
    arr = C.c_void_p * n
    parts = arr(*[ptr(e[0]) for e in entries])
    dgs = arr(*[ptr(e[1]) for e in entries])
    dbs = arr(*[ptr(e[2]) for e in entries])
    call("kdfm_ln_fold", C.cast(parts, C.POINTER(C.c_void_p)), C.cast(dgs, C.POINTER(C.c_void_p)),
         C.cast(dbs, C.POINTER(C.c_void_p)), n, rows, d, _s())


def qkv_prep(qkv, u, v, qu, qv):
    rows, d = qu.shape
    assert qkv.shape == (rows, 3 * d) and u.numel() == d and v.numel() == d
    call("kdfm_qkv_prep", ptr(qkv), ptr(u), ptr(v), ptr(qu), ptr(qv), rows, d, _s())


ATTN_BWD_ROWDOT, ATTN_BWD_DQ, ATTN_BWD_DKV, ATTN_BWD_DPOS, ATTN_BWD_ALL = 1, 2, 4, 8, 15


def relpos_attn_bwd_ws(B, H, T, d):
    return int(_lib.lib().kdfm_relpos_attn_bwd_ws(B, H, T, d))


def attn_saved(B, H, T, device):
    """The single-pass forward's saved operands for the backward: lse (B,H,T) f32, p~ (B,H,T,T) bf16 and
    the per-64-key-block running maxima m_blk (B,H,T,ceil(T/64)) f32."""
    return (torch.empty(B, H, T, device=device), torch.empty(B, H, T, T, dtype=torch.bfloat16, device=device),
            torch.empty(B, H, T, (T + 63) // 64, device=device))


def relpos_attn_bwd(do, o, qu, qv, qkv, ppos, lse, p_tilde, m_blk, lengths, dqu, dqv, dqkv, dppos, B, H, T, scale, p,
                    seed, rng_stream, parts=ATTN_BWD_ALL, ws=None):
    """Fused attention backward (csrc/attn_bwd.hip): dqu, dqv, dK/dV into dqkv[:, d:], dppos.  DQ
    recomputes the probabilities from the forward's per-row log-sum-exp `lse` (B, H, T); DKV / DPOS form
    them from the forward's bf16 `p_tilde` and block maxima `m_blk` (attn_saved).  `parts` (ATTN_BWD_*)
    issues a subset; parts issued on different streams must share a dedicated `ws`
    (relpos_attn_bwd_ws floats) and be ordered after ROWDOT."""
    rows, d = do.shape
    assert rows == B * T and qkv.shape == (rows, 3 * d) and lse.shape == (B, H, T)
    if parts & (ATTN_BWD_DKV | ATTN_BWD_DPOS):
        assert p_tilde is not None and p_tilde.dtype == torch.bfloat16 and p_tilde.shape == (B, H, T, T)
        assert m_blk is not None and m_blk.shape == (B, H, T, (T + 63) // 64)
    assert dppos is None or dppos.shape == (2 * T - 1, d)
    for t in (do, o, qu, qv, qkv, ppos, lse, p_tilde, m_blk, dqu, dqv, dqkv, dppos):
        assert t is None or t.is_contiguous()
    assert o.shape == do.shape
    if parts != ATTN_BWD_ALL:
        assert ws is not None and ws.numel() >= relpos_attn_bwd_ws(B, H, T, d)
        # algorithmic work of the issued parts (per (b, h), 2 T^2 dk FLOP per product): DQ recomputes the
        # scores (QK^T + band) and forms dP, dQu, dQv; DKV dP, dK, dV; DPOS dP and dPpos.  Bytes: the row
        # operands each part reads / writes once at f32, p~ (bf16) once per part that reads it
        dk = d // H
        tt = 2.0 * B * H * T * T * dk
        fl = tt * ((5 if parts & ATTN_BWD_DQ else 0) + (3 if parts & ATTN_BWD_DKV else 0)
                   + (2 if parts & ATTN_BWD_DPOS else 0))
        nrow = (2 if parts & ATTN_BWD_ROWDOT else 0) + (6 if parts & ATTN_BWD_DQ else 0) + \
            (6 if parts & ATTN_BWD_DKV else 0) + (3 if parts & ATTN_BWD_DPOS else 0)
        nb = 4.0 * rows * d * nrow + 2.0 * B * H * T * T * ((1 if parts & ATTN_BWD_DKV else 0)
                                                            + (1 if parts & ATTN_BWD_DPOS else 0))
        _traced("attn_bwd", fl, nb, "kdfm_relpos_attn_bwd_parts", ptr(do), ptr(o), ptr(qu), ptr(qv), ptr(qkv),
                ptr(ppos), ptr(lse), ptr(p_tilde), ptr(m_blk), ptr(_i64(lengths)), ptr(dqu), ptr(dqv), ptr(dqkv),
                ptr(dppos), ptr(ws), ws.numel(), B, H, T, d, float(scale), float(p), ptr(seed), int(rng_stream),
                int(parts), _s())
        return
    ws = scratch(do.device, relpos_attn_bwd_ws(B, H, T, d))
    # algorithmic: per (b, h) the products dP (twice: DQ and DKV / DPOS), dQu, dQv, dK, dV, dPpos (2 T^2 dk
    # each, the positional band counted as one T x T) plus DQ's score recompute (QK^T + band); bytes: dO, O,
    # qu, qv, K, V read once, dqu, dqv, dK, dV written, lse read, p~ read twice (DKV, DPOS)
    dk = d // H
    fl = 2.0 * B * H * T * T * dk * 9
    nb = 4.0 * rows * d * 10 + 4.0 * B * H * T + 2.0 * 2.0 * B * H * T * T
    _traced("attn_bwd", fl, nb, "kdfm_relpos_attn_bwd", ptr(do), ptr(o), ptr(qu), ptr(qv), ptr(qkv), ptr(ppos),
            ptr(lse), ptr(p_tilde), ptr(m_blk), ptr(_i64(lengths)), ptr(dqu), ptr(dqv), ptr(dqkv), ptr(dppos),
            ptr(ws), ws.numel(), B, H, T, d, float(scale), float(p), ptr(seed), int(rng_stream), _s())


def attn_bwd2_saved(B, H, T, device):
    """bwd2's saved T x T operands, written by relpos_attn_bwd2_dq: dS and Pd, each (B, H, T, ldt) bf16."""
    ldt = int(_lib.lib().kdfm_relpos_attn_bwd2_ldt(T))
    return (torch.empty(B, H, T, ldt, dtype=torch.bfloat16, device=device),
            torch.empty(B, H, T, ldt, dtype=torch.bfloat16, device=device))


def relpos_attn_bwd2_dq(do, o, qu, qv, qkv, ppos, lse, lengths, rsum, ds, pd, dqu, dqv, B, H, T, scale, p, seed,
                        rng_stream):
    """bwd2 part 1 (csrc/attn_bwd.hip): dqu / dqv (the row sums r_i = dO_i . O_i formed in-kernel; rsum is
    unused and may be None), and the bf16
    dS / Pd (attn_bwd2_saved) the _dkv / _dpos parts read."""
    rows, d = do.shape
    assert rows == B * T and qkv.shape == (rows, 3 * d) and lse.shape == (B, H, T) and o.shape == do.shape
    assert ds.dtype == torch.bfloat16 and pd.dtype == torch.bfloat16
    assert ds.shape == pd.shape and ds.shape[:3] == (B, H, T) and ds.is_contiguous() and pd.is_contiguous()
    for t in (do, o, qu, qv, qkv, ppos, lse, dqu, dqv):
        assert t.is_contiguous()
    dk = d // H
    tt = 2.0 * B * H * T * T * dk
    # scores (QK^T + band), dP, dQu, dQv: 5 T x T products; bytes: dO, O, qu, qv, K, V read, dqu, dqv written,
    # dS and Pd written (bf16)
    _traced("attn_bwd", 5 * tt, 4.0 * rows * d * 8 + 2.0 * 2.0 * B * H * T * T, "kdfm_relpos_attn_bwd2_dq", ptr(do),
            ptr(o), ptr(qu), ptr(qv), ptr(qkv), ptr(ppos), ptr(lse), ptr(_i64(lengths)), ptr(rsum), ptr(ds), ptr(pd),
            ptr(dqu), ptr(dqv), B, H, T, d, float(scale), float(p), ptr(seed), int(rng_stream), _s())


def relpos_attn_bwd2_dq3(do, o, qu, qv, prep, pband, lse, lengths, ds, pd, dqu, dqv, B, H, T, scale, p, seed,
                         rng_stream):
    """bwd2 part 1 over the forward's prepared operands (attn_kv_prep's triple and this layer's attn_band_prep
    slice, kdfm_relpos_attn_bwd2_dq3): the same outputs as relpos_attn_bwd2_dq."""
    rows, d = do.shape
    kb, vb, cen = prep
    assert rows == B * T and lse.shape == (B, H, T) and o.shape == do.shape
    assert ds.dtype == torch.bfloat16 and pd.dtype == torch.bfloat16
    assert ds.shape == pd.shape and ds.shape[:3] == (B, H, T) and ds.is_contiguous() and pd.is_contiguous()
    for t in (do, o, qu, qv, lse, dqu, dqv):
        assert t.is_contiguous()
    tt = 2.0 * B * H * T * T * (d // H)
    # scores (QK^T + band), dP, dQu, dQv: 5 T x T products; bytes: dO, O, qu, qv read, dqu, dqv written (f32), the
    # bf16 K / V images read, dS and Pd written (bf16)
    _traced("attn_bwd", 5 * tt, 4.0 * rows * d * 6 + 2.0 * 2 * kb.numel() + 2.0 * 2.0 * B * H * T * T,
            "kdfm_relpos_attn_bwd2_dq3", ptr(do), ptr(o), ptr(qu), ptr(qv), ptr(kb), ptr(vb), ptr(cen), ptr(pband),
            ptr(lse), ptr(_i64(lengths)), ptr(ds), ptr(pd), ptr(dqu), ptr(dqv), B, H, T, d, float(scale), float(p),
            ptr(seed), int(rng_stream), _s())


def relpos_attn_bwd2_dkv(do, qu, ds, pd, lengths, dqkv, B, H, T):
    """bwd2 part 2: dK / dV into dqkv[:, d:] / [:, 2d:] from the saved dS / Pd (no recompute)."""
    rows, d = do.shape
    assert dqkv.shape == (rows, 3 * d) and dqkv.is_contiguous() and do.is_contiguous() and qu.is_contiguous()
    tt = 2.0 * B * H * T * T * (d // H)
    _traced("attn_bwd", 2 * tt, 4.0 * rows * d * 4 + 2.0 * 2.0 * B * H * T * T, "kdfm_relpos_attn_bwd2_dkv", ptr(do),
            ptr(qu), ptr(ds), ptr(pd), ptr(_i64(lengths)), ptr(dqkv), B, H, T, d, _s())


def relpos_attn_bwd2_dpos_ws(B, T, d):
    return int(_lib.lib().kdfm_relpos_attn_bwd2_dpos_ws(B, T, d))


def relpos_attn_bwd2_dpos(qv, ds, lengths, dppos, B, H, T, ws=None):
    """bwd2 part 3: dppos (2T-1, d) from the saved dS and qv (ordered per-utterance-chunk fold)."""
    rows, d = qv.shape
    assert dppos.shape == (2 * T - 1, d) and dppos.is_contiguous() and qv.is_contiguous()
    n = relpos_attn_bwd2_dpos_ws(B, T, d)
    if ws is None:
        ws = scratch(qv.device, n)
    assert ws.numel() >= n
    tt = 2.0 * B * H * T * T * (d // H)
    _traced("attn_bwd", tt, 4.0 * rows * d + 2.0 * B * H * T * T + 4.0 * (2 * T - 1) * d,
            "kdfm_relpos_attn_bwd2_dpos", ptr(qv), ptr(ds), ptr(_i64(lengths)), ptr(dppos), ptr(ws), ws.numel(), B, H,
            T, d, _s())


def relpos_attn_fwd(qu, qv, qkv, ppos, lengths, o, P, Pd, B, H, T, scale, p, seed, rng_stream, lse=None, p_tilde=None,
                    m_blk=None):
    """Fused rel-pos MHA forward (bf16): P / Pd (B,H,T,T) written when given (two passes), else one
    online-softmax pass that writes the per-row log-sum-exp `lse` (B,H,T) and the backward's bf16
    p~ / block maxima (attn_saved) when given."""
    rows, d = qu.shape
    assert rows == B * T and qkv.shape == (rows, 3 * d) and ppos.shape == (2 * T - 1, d) and o.shape == (rows, d)
    assert qu.is_contiguous() and qv.is_contiguous() and qkv.is_contiguous() and ppos.is_contiguous()
    assert lse is None or (lse.shape == (B, H, T) and P is None and Pd is None)
    assert (p_tilde is None) == (m_blk is None)
    if p_tilde is not None:
        assert lse is not None and p_tilde.dtype == torch.bfloat16 and p_tilde.shape == (B, H, T, T)
        assert m_blk.shape == (B, H, T, (T + 63) // 64) and p_tilde.is_contiguous() and m_blk.is_contiguous()
    # algorithmic: QK^T, the positional band (one T x T-equivalent) and PV, 2 T^2 dk FLOP each per (b, h);
    # bytes: qu, qv, K, V, o once (+ P written when saved, + lse, + p~ bf16)
    fl = 2.0 * B * H * T * T * (d // H) * 3
    nb = 4.0 * rows * d * 5 + (4.0 * B * H * T * T if P is not None else 0.0) + (4.0 * B * H * T if lse is not None
                                                                                 else 0.0)
    nb += 2.0 * B * H * T * T if p_tilde is not None else 0.0
    _traced("attn_fwd", fl, nb, "kdfm_relpos_attn_fwd", ptr(qu), ptr(qv), ptr(qkv), ptr(ppos), ptr(_i64(lengths)),
            ptr(o), ptr(P), ptr(Pd), ptr(lse), ptr(p_tilde), ptr(m_blk), B, H, T, d, float(scale), float(p), ptr(seed),
            rng_stream, _s())


def attn_kv_prep(qkv, lengths, B, H, T, out=None):
    """The bf16 centred key / value tiles and the centre of kdfm_relpos_attn_fwd3 (csrc/attn_fwd3.hip):
    returns (kb, vb, centre); `out` reuses a previous triple of the same shape."""
    rows, d3 = qkv.shape
    d = d3 // 3
    assert rows == B * T and qkv.is_contiguous() and qkv.dtype == torch.float32
    n = int(_lib.lib().kdfm_attn_kv_prep_elems(B, H, T, d))
    nc = int(_lib.lib().kdfm_attn_centre_elems(B, H, d))
    if n < 0 or nc < 0:
        raise _lib.KdfmError(f"attn_kv_prep: unsupported d={d} H={H}")
    if out is None:
        out = (torch.empty(n, dtype=torch.bfloat16, device=qkv.device),
               torch.empty(n, dtype=torch.bfloat16, device=qkv.device), torch.empty(nc, device=qkv.device))
    kb, vb, cen = out
    assert kb.numel() >= n and vb.numel() >= n and cen.numel() >= nc
    # read K, V (f32) once, write the two bf16 images (padded rows / columns)
    _traced("attn_prep", 0.0, 4.0 * rows * 2 * d + 2.0 * 2 * n, "kdfm_attn_kv_prep", ptr(qkv), ptr(_i64(lengths)),
            ptr(kb), ptr(vb), ptr(cen), B, H, T, d, _s())
    return out


def attn_band_prep(pos, H, T, out=None):
    """Every layer's projected positions pos (layers, 2T-1, d) (or one layer's (2T-1, d)) as the bf16 band rows
    of kdfm_relpos_attn_fwd3: returns pb (layers, H * NPB * LR) -- pb[l] is layer l's slice."""
    if pos.dim() == 2:
        pos = pos.unsqueeze(0)
    L, npos, d = pos.shape
    assert npos == 2 * T - 1 and pos.stride(2) == 1 and pos.stride(1) == d and pos.dtype == torch.float32
    n = int(_lib.lib().kdfm_attn_band_prep_elems(1, H, T, d))
    if n < 0:
        raise _lib.KdfmError(f"attn_band_prep: unsupported d={d} H={H}")
    if out is None:
        out = torch.empty(L, n, dtype=torch.bfloat16, device=pos.device)
    assert out.shape[0] >= L and out.shape[1] == n and out.is_contiguous()
    _traced("attn_prep", 0.0, 4.0 * L * npos * d + 2.0 * L * n, "kdfm_attn_band_prep", ptr(pos),
            pos.stride(0) if L > 1 else npos * d, L, ptr(out), H, T, d, _s())
    return out


def relpos_attn_fwd3(qu, qv, prep, pband, lengths, o, B, H, T, scale, p, seed, rng_stream, lse=None):
    """kdfm_relpos_attn_fwd3: the single-pass fused forward over the prepared operands (attn_kv_prep's triple,
    one layer's attn_band_prep slice); O / lse bitwise relpos_attn_fwd's single pass."""
    rows, d = qu.shape
    kb, vb, cen = prep
    assert rows == B * T and o.shape == (rows, d) and qu.is_contiguous() and qv.is_contiguous()
    assert lse is None or lse.shape == (B, H, T)
    assert pband.dtype == torch.bfloat16 and pband.numel() == int(_lib.lib().kdfm_attn_band_prep_elems(1, H, T, d))
    # algorithmic: QK^T, the positional band (one T x T-equivalent) and PV per (b, h); bytes: qu, qv, o (f32) and
    # the bf16 key / value images once (+ lse)
    fl = 2.0 * B * H * T * T * (d // H) * 3
    nb = 4.0 * rows * d * 3 + 2.0 * 2 * kb.numel() + (4.0 * B * H * T if lse is not None else 0.0)
    _traced("attn_fwd", fl, nb, "kdfm_relpos_attn_fwd3", ptr(qu), ptr(qv), ptr(kb), ptr(vb), ptr(cen), ptr(pband),
            ptr(_i64(lengths)), ptr(o), ptr(lse), B, H, T, d, float(scale), float(p), ptr(seed), int(rng_stream), _s())


def relpos_softmax_fwd(ac, bd, lengths, P, Pd, B, H, T, scale, p, seed, rng_stream):
    assert ac.numel() == B * H * T * T and bd.numel() == B * H * T * (2 * T - 1)
    call("kdfm_relpos_softmax_fwd", ptr(ac), ptr(bd), ptr(_i64(lengths)), ptr(P), ptr(Pd), B, H, T, float(scale),
         float(p), ptr(seed), int(rng_stream), _s())


def relpos_softmax_bwd(P, dPd, dAC, dBD, B, H, T, scale, p, seed, rng_stream):
    assert dBD.numel() == B * H * T * (2 * T - 1)
    call("kdfm_relpos_softmax_bwd", ptr(P), ptr(dPd), ptr(dAC), ptr(dBD), B, H, T, float(scale), float(p), ptr(seed),
         int(rng_stream), _s())


def glu_mask_fwd(a, lengths, g, B, T, d):
    call("kdfm_glu_mask_fwd", ptr(a), ptr(_i64(lengths)), ptr(g), B, T, d, _s())


def glu_mask_bwd(dg, a, lengths, da, B, T, d):
    """da f32, or bf16 (rounded to nearest even)."""
    if da.dtype == torch.bfloat16:
        call("kdfm_glu_mask_bwd_bf16", ptr(dg), ptr(a), ptr(_i64(lengths)), da.data_ptr(), B, T, d, _s())
        return
    call("kdfm_glu_mask_bwd", ptr(dg), ptr(a), ptr(_i64(lengths)), ptr(da), B, T, d, _s())


def dwconv_fwd(g, w, bias, y, stats, B, T, d, K):
    call("kdfm_dwconv_fwd", ptr(g), ptr(w), ptr(bias), ptr(y), ptr(stats), B, T, d, K, _s())


def dwconv_bwd(dy, g, w, dg, dw, db, B, T, d, K, *, ws=None):
    """dg = conv^T(dy) and dw / db (+=).  dw = db = None with `ws` given: only dg, the weight-gradient
    partials left in ws for dwconv_bwd_fold (e.g. on another stream)."""
    if ws is None:
        assert dw is not None
        ws = scratch(dy.device, _lib.lib().kdfm_dwconv_bwd_ws(B, T, d, K))
    call("kdfm_dwconv_bwd", ptr(dy), ptr(g), ptr(w), ptr(dg), ptr(dw), ptr(db), ptr(ws), B, T, d, K, _s())


def dwconv_bwd_bn(dz, y, mean, rstd, gamma, beta, red, red_next, dgamma, dbeta, batch_stats, g, w, dg, ws, B, T, d,
                  K):
    """Depthwise backward with the BatchNorm(+SiLU) backward's elementwise half applied on load
    (kdfm_dwconv_bwd_bn): dz = d loss / d silu(BN(y)), red = the bn_silu_bwd_reduce sums; leaves the weight
    partials in ws (dwconv_bwd_fold) and adds the BN affine gradients."""
    call("kdfm_dwconv_bwd_bn", ptr(dz), ptr(y), ptr(mean), ptr(rstd), ptr(gamma), ptr(beta), ptr(red), ptr(red_next),
         ptr(dgamma), ptr(dbeta), int(batch_stats), ptr(g), ptr(w), ptr(dg), ptr(ws), B, T, d, K, _s())


def bn_silu_bwd_reduce(dz, y, mean, rstd, gamma, beta, red):
    rows, d = y.shape
    call("kdfm_bn_silu_bwd_reduce", ptr(dz), ptr(y), ptr(mean), ptr(rstd), ptr(gamma), ptr(beta), ptr(red), rows, d,
         _s())


def dwconv_bwd_ws(B, T, d, K):
    return int(_lib.lib().kdfm_dwconv_bwd_ws(B, T, d, K))


def dwconv_bwd_fold(ws, dw, db, B, T, d, K):
    call("kdfm_dwconv_bwd_fold", ptr(ws), ptr(dw), ptr(db), B, T, d, K, _s())


def bn_finalize(stats, rm, rv, mean, rstd, d, count, eps):
    call("kdfm_bn_finalize", ptr(stats), ptr(rm), ptr(rv), ptr(mean), ptr(rstd), d, int(count), float(eps), _s())


def bn_running_update(rm, rv, stats, d, count, momentum):
    call("kdfm_bn_running_update", ptr(rm), ptr(rv), ptr(stats), d, int(count), float(momentum), _s())


def bn_finalize_running(stats, rm, rv, mean, rstd, d, count, eps, momentum):
    """Batch mean/rstd from the f64 sums AND the running-statistics update (training), one launch."""
    call("kdfm_bn_finalize_running", ptr(stats), ptr(rm), ptr(rv), ptr(mean), ptr(rstd), d, int(count), float(eps),
         float(momentum), _s())


def bn_silu_fwd(y, mean, rstd, g, b, z):
    """z f32, or bf16 (rounded to nearest even)."""
    rows, d = y.shape
    if z.dtype == torch.bfloat16:
        call("kdfm_bn_silu_fwd_bf16", ptr(y), ptr(mean), ptr(rstd), ptr(g), ptr(b), z.data_ptr(), rows, d, _s())
        return
    call("kdfm_bn_silu_fwd", ptr(y), ptr(mean), ptr(rstd), ptr(g), ptr(b), ptr(z), rows, d, _s())


def bn_silu_bwd(dz, y, mean, rstd, g, b, red_ws, dy, dg, db, batch_stats=True, red_next=None, zeroed=False):
    """zeroed: red_ws is already zero (no memset; kdfm_bn_silu_bwd2), and red_next (when given) is zeroed by the
    launch for the next call."""
    rows, d = y.shape
    if zeroed:
        call("kdfm_bn_silu_bwd2", ptr(dz), ptr(y), ptr(mean), ptr(rstd), ptr(g), ptr(b), ptr(red_ws), ptr(red_next),
             ptr(dy), ptr(dg), ptr(db), rows, d, int(batch_stats), _s())
        return
    call("kdfm_bn_silu_bwd", ptr(dz), ptr(y), ptr(mean), ptr(rstd), ptr(g), ptr(b), ptr(red_ws), ptr(dy), ptr(dg),
         ptr(db), rows, d, int(batch_stats), _s())


# ------------------------------------------------------------------------------------------------
# losses / heads / optimizer
# ------------------------------------------------------------------------------------------------

def log_softmax(x, y):
    rows, Cc = x.shape
    call("kdfm_log_softmax", ptr(x), ptr(y), rows, Cc, x.stride(0), y.stride(0), _s())


def argmax_rows(x, idx):
    rows, Cc = x.shape
    assert x.is_contiguous() and idx.dtype == torch.int64 and idx.numel() == rows
    call("kdfm_argmax_rows", ptr(x), ptr(idx), rows, Cc, _s())


def log_softmax_bwd(dy, y, dx):
    rows, Cc = y.shape
    assert dy.is_contiguous() and y.is_contiguous() and dx.is_contiguous()
    call("kdfm_log_softmax_bwd", ptr(dy), ptr(y), ptr(dx), rows, Cc, _s())


def ctc_loss(lp, targets, in_len, tgt_len, alpha_ws, beta_ws, nll, grad, B, T, Cc, blank, grad_scale,
             zero_infinity=True):
    Umax = targets.shape[1]
    assert targets.dtype == torch.int64 and targets.is_contiguous()
    assert alpha_ws.numel() >= B * T * (2 * Umax + 1) and beta_ws.numel() >= B * T * (2 * Umax + 1)
    call("kdfm_ctc_loss", ptr(lp), ptr(targets), ptr(_i64(in_len)), ptr(_i64(tgt_len)), ptr(alpha_ws), ptr(beta_ws),
         ptr(nll), ptr(grad), B, T, Cc, Umax, blank, float(grad_scale), int(zero_infinity), _s())


def kl_div_logits(lp, tlogits, grad, loss_acc, temperature, grad_coef, loss_scale):
    rows, Cc = lp.shape
    call("kdfm_kl_div_logits", ptr(lp), ptr(tlogits), ptr(grad), ptr(loss_acc), rows, Cc, float(temperature),
         float(grad_coef), float(loss_scale), _s())


def loss_combine(nll, kl, recon, fm, kd_alpha, out5):
    call("kdfm_loss_combine", ptr(nll), nll.numel(), ptr(kl), ptr(recon), ptr(fm), float(kd_alpha), ptr(out5), _s())


def adapter_fwd(zs, h, w2, b2, eps_in, zn, gamma, seed, rng_stream):
    rows, L = zs.shape
    call("kdfm_adapter_fwd", ptr(zs), ptr(h), ptr(w2), ptr(b2), ptr(eps_in), ptr(zn), ptr(gamma), rows, L, ptr(seed),
         int(rng_stream), _s())


def adapter_bwd(dzn, zs, h, gamma, w2, eps_in, dzs, dh, dw2, db2, seed, rng_stream):
    rows, L = zs.shape
    ws = scratch(zs.device, int(_lib.lib().kdfm_adapter_bwd_ws(rows, L)))
    call("kdfm_adapter_bwd", ptr(dzn), ptr(zs), ptr(h), ptr(gamma), ptr(w2), ptr(eps_in), ptr(dzs), ptr(dh),
         ptr(dw2), ptr(db2), ptr(ws), ws.numel(), rows, L, ptr(seed), int(rng_stream), _s())


def fm_step_bias(w_te, b_te, W1, b1, cvec, evec, L, E, steps):
    call("kdfm_fm_step_bias", ptr(w_te), ptr(b_te), ptr(W1), ptr(b1), ptr(cvec), ptr(evec), L, E, steps, _s())


def fm_time_bwd(dc, evec, W1, dW1, db1, dw_te, db_te, L, E, steps):
    call("kdfm_fm_time_bwd", ptr(dc), ptr(evec), ptr(W1), ptr(dW1), ptr(db1), ptr(dw_te), ptr(db_te), L, E, steps,
         _s())


def adamw_noam(p, g, m, v, step, base_lr, d_model, warmup, min_lr, beta1, beta2, eps, wd, grad_scale, lr_out=None,
               adam_base=None, gstats=None, p16=None):
    """Fused AdamW + Noam (csrc/optim.hip); with `gstats` (grad_stats' output) the update is skipped
    when the gradient holds a non-finite value.  p16: the flat buffer's bf16 mirror, written in the same pass."""
    assert p.numel() == g.numel() == m.numel() == v.numel()
    assert gstats is None or (gstats.numel() >= 2 and gstats.dtype == torch.float32)
    if p16 is not None:
        assert p16.numel() == p.numel() and p16.dtype == torch.bfloat16
        call("kdfm_adamw_noam_bf16", ptr(p), ptr(g), ptr(m), ptr(v), p16.data_ptr(), p.numel(), ptr(step),
             ptr(adam_base), float(base_lr), float(d_model), float(warmup), float(min_lr), float(beta1), float(beta2),
             float(eps), float(wd), float(grad_scale), ptr(lr_out), ptr(gstats), _s())
        return
    call("kdfm_adamw_noam", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(step), ptr(adam_base), float(base_lr),
         float(d_model),
         float(warmup), float(min_lr), float(beta1), float(beta2), float(eps), float(wd), float(grad_scale),
         ptr(lr_out), ptr(gstats), _s())


def grad_stats(g, scale, out2):
    """out2 = [sum (scale g)^2 over finite entries, number of non-finite entries] (deterministic)."""
    assert g.is_contiguous() and g.dtype == torch.float32 and out2.numel() >= 2
    n = int(_lib.lib().kdfm_grad_stats_ws())
    ws = scratch(g.device, n)
    call("kdfm_grad_stats", ptr(g), g.numel(), float(scale), ptr(ws), ws.numel(), ptr(out2), _s())
