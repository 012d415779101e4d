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


def max_over_ranks(value: float, device) -> float:
    """Max of a host float over all ranks (bench timing: the slowest rank defines the step)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
