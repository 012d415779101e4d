"""Weight-gradient overlap: run the backward's weight-gradient GEMMs on a second HIP stream.

In the backward every Linear contributes a dX product (on the critical path: the next layer needs
it) and a dW product (needed only by the optimizer).  The dW GEMMs of the Conformer layers are
small (K = B*T' rows, a few hundred outputs) and latency bound, so running them concurrently
with the dX chain fills CUs the chain leaves idle.  Ordering:

  * fork: the side stream waits for everything issued on the main stream so far (one event), so
    the dY / X operands are complete;
  * the operand tensors are kept referenced until the join, so the caching allocator cannot hand
    their memory to main-stream work while the side stream still reads them (capture-safe,
    unlike record_stream);
  * join: the main stream waits for the side stream before anything reads the accumulated
    gradients (optimizer, all-reduce, or a consumer of a side-produced partial).

Both streams are captured into the same HIP graph by GraphedTrainStep (fork/join are graph
edges)."""
from __future__ import annotations

import os

import torch

from . import kernels as K

# KDFM_WGRAD_CUS=n: the weight-gradient stream is created restricted to n CUs (spread over every XCD;
# kdfm_stream_create_cu_mask), so its products never hold every CU's LDS / wave slots when the
# critical-path kernels arrive; the row-parallel weight gradients then target n workgroups (fewer
# K-splits, smaller partials) unless KDFM_WGR_WGS says otherwise.  0 (default): an ordinary stream.
WGRAD_CUS = int(os.environ.get("KDFM_WGRAD_CUS", "0"))
if WGRAD_CUS > 0:
    os.environ.setdefault("KDFM_WGR_WGS", str(WGRAD_CUS))


def _masked_stream(dev, n_cus):
    import ctypes as C

    from . import _lib
    with torch.cuda.device(dev):
        out = C.c_void_p()
        _lib.check(_lib.lib().kdfm_stream_create_cu_mask(int(n_cus), C.byref(out)), "kdfm_stream_create_cu_mask")
        return torch.cuda.ExternalStream(out.value, device=dev)


class WgradOverlap:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self._side = {}
        self._links = {}
        self._keep = []
        self._pending = False

    def _stream(self, dev):
        key = torch.device(dev).index if not isinstance(dev, int) else dev
        s = self._side.get(key)
        if s is None:
            s = _masked_stream(key, WGRAD_CUS) if WGRAD_CUS > 0 else torch.cuda.Stream(device=key)
            self._side[key] = s
            self._links[key] = (K.StreamLink(), K.StreamLink())
        return s

    def run(self, fn, *keep):
        """Issue fn() (kernel launches only) on the side stream after all current main-stream work."""
        if not self.enabled:
            fn()
            return
        dev = K.current_device()
        side = self._stream(dev)
        self._links[dev][0].after_current(side)
        with K.on_stream(side):
            fn()
        self._keep.extend(keep)
        self._pending = True

    def stream(self):
        """The side stream of the current device (created on first use).  The engine also borrows it in
        the forward, where no weight gradient runs, for the first layer-half of the KD heads."""
        return self._stream(K.current_device())

    def stream_after_current(self):
        """The side stream, ordered after all current main-stream work (None when weight gradients run
        in line): the bucketed all-reduce issues its collectives from it, so they start after both the
        main stream's and the side stream's gradient work without a stream of their own."""
        if not self.enabled:
            return None
        dev = K.current_device()
        side = self._stream(dev)
        self._links[dev][0].after_current(side)
        return side

    def fence(self, stream) -> None:
        """`stream` waits for every side-stream launch issued so far (no effect when none pending)."""
        if self._pending:
            K.wait_stream(stream, self._stream(stream.device))

    def serialized(self, on: bool = True):
        """Context manager: with on=True every weight-gradient product runs in line on the issuing
        stream (deterministic mode: bitwise-reproducible backward, see engine.Ver5Engine._mode)."""
        ov = self

        class _Ctx:
            def __enter__(self):
                self.prev = ov.enabled
                if on:
                    ov.join()
                    ov.enabled = False
                return self

            def __exit__(self, *a):
                ov.enabled = self.prev

        return _Ctx()

    def join(self):
        """Main stream waits for all side-stream work; releases the kept operands."""
        if not self._pending:
            return
        dev = K.current_device()
        self._links[dev][1].current_after(self._stream(dev))
        self._keep.clear()
        self._pending = False


WGRAD = WgradOverlap()
