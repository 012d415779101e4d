"""Data-parallel gradient exchange for the ver5 step.

One process per GPU; each rank trains on its own B=32 shard (no data-path collective), then the
ONE flat gradient buffer of all trainable parameters (3.44M fp32 = 13.8 MB) is summed with a single
RCCL all-reduce over xGMI (torch.distributed backend "nccl" is RCCL on ROCm) and the fused AdamW
applies the 1/world mean.  A flat buffer makes the exchange one large collective instead of ~600
per-parameter calls (the reference's Lightning DDP default would bucket per 25 MB and would error on
the unused fm_latent_2 parameters, SURVEY.md §0.7 - they are simply not part of the buffer here).
BatchNorm statistics stay per rank, as in the reference (no sync_batchnorm).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class FlatGradAllReduce:
    """Callable used by Ver5Engine.train_step / GraphedTrainStep: sums the flat gradient buffer
    across ranks in `buckets` contiguous chunks (1 = one collective) and returns the mean scale."""

    def __init__(self, group=None, buckets: int = 1):
        self.group = group
        self.world = dist.get_world_size(group)
        self.buckets = max(1, int(buckets))

    def __call__(self, flat: torch.Tensor) -> float:
        if self.world == 1:
            return 1.0
        if self.buckets == 1:
            dist.all_reduce(flat, group=self.group)
        else:
            for chunk in flat.chunk(self.buckets):
                dist.all_reduce(chunk, group=self.group)
        return 1.0 / self.world


class BucketedGradAllReduce:
    """Bucketed all-reduce overlapped with the backward (2-4 buckets in reverse
    layer order, each launched as soon as its gradients are final).

    The flat gradient buffer is laid out encoder (subsampling, layers 0..15), decoder, heads, and the
    backward finalises it from the END: heads, then the decoder, then layers 15..0, then the
    subsampling.  Ver5Engine.backward calls `ready(flat, offset)` whenever every gradient at index
    >= offset is final (after the heads, the decoder, every encoder layer); each bucket
    [lo, hi) with lo >= offset that has not been launched yet is all-reduced asynchronously, issued
    from the weight-gradient side stream (kdfm.overlap.WGRAD) after it has joined the main stream, so
    the collective -- on RCCL's own stream, which waits for the issuing one -- starts once both
    streams' gradients for the bucket are final, and RCCL over xGMI runs while the dX chain of the
    lower layers continues.  No extra stream of ours: compute, teacher (+ CTC/KL), weight gradients
    and RCCL's stream are four, one per hardware queue (GPU_MAX_HW_QUEUES=4).  With weight gradients
    in line (deterministic mode) the collective is issued from the main stream.
    `__call__(flat)` (after the backward) launches what is left, makes the current stream wait for
    every collective and returns the 1/world mean scale for the fused AdamW.  With no ready() calls
    it is exactly FlatGradAllReduce with `buckets` chunks.  Bucket edges are aligned to 64 floats."""

    def __init__(self, numel: int, group=None, buckets: int = 4, force: bool = False):
        """force: issue the collectives even in a world of one rank (they are then identities) -- test-only, so
        the RCCL path (its own stream ordered behind the issuing one, Work.wait() as a device-side wait, a step
        plan's replay of the ready() callbacks) runs on a one-GPU box (tests/test_rccl_gpu.py)."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.active = self.world > 1 or force
        self.issued = 0   # collectives issued so far (tests count them)
        nb = max(1, int(buckets))
        step = -(-numel // nb)
        step = -(-step // 64) * 64
        self.edges = [min(numel, i * step) for i in range(nb)] + [numel]
        self.edges = sorted(set(self.edges))
        self._works = []
        self._launched = set()

    def _launch(self, flat, k: int):
        lo, hi = self.edges[k], self.edges[k + 1]
        side = None
        if flat.is_cuda:
            from .overlap import WGRAD
            side = WGRAD.stream_after_current()
        if side is None:
            self._works.append(self._issue(flat[lo:hi], k))
        else:
            with torch.cuda.stream(side):
                self._works.append(self._issue(flat[lo:hi], k))
        self._launched.add(k)

    def _issue(self, chunk: torch.Tensor, k: int):
        """The collective of bucket k, issued on the current (issuing) stream; returns its work handle."""
        self.issued += 1
        return dist.all_reduce(chunk, group=self.group, async_op=True)

    def ready(self, flat: torch.Tensor, offset: int) -> None:
        if not self.active:
            return
        for k in range(len(self.edges) - 2, -1, -1):
            if k not in self._launched and self.edges[k] >= offset:
                self._launch(flat, k)

    def __call__(self, flat: torch.Tensor) -> float:
        if not self.active:
            return 1.0
        for k in range(len(self.edges) - 2, -1, -1):
            if k not in self._launched:
                self._launch(flat, k)
        for w in self._works:
            if w is not None:
                w.wait()   # device-side: the current stream waits for the collective
        self._works.clear()
        self._launched.clear()
        return 1.0 / self.world


def max_over_ranks(value: float, device) -> float:
    """Max of a host float over all ranks (bench timing: the slowest rank defines the step)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
