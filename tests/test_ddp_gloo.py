"""World-size-2 gloo tests (CPU) of the data-parallel path: the flat-gradient all-reduce sums rank
shards and yields the DDP mean scale; max-over-ranks timing picks the slowest rank."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, buckets, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))
    from kdfm.ddp import FlatGradAllReduce, max_over_ranks
    n = 3_438_090  # trainable parameters of the ver5 step
    g = torch.full((n,), float(rank + 1))
    g[::7] = rank * 10.0
    ar = FlatGradAllReduce(buckets=buckets)
    scale = ar(g)
    t = max_over_ranks(1.5 + rank, torch.device("cpu"))
    out[rank] = (float(g[1]), float(g[0]), scale, t)
    dist.destroy_process_group()


def _run(buckets):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), buckets, out), nprocs=world, join=True)
    for r in range(world):
        s1, s0, scale, t = out[r]
        assert s1 == 3.0          # 1 + 2
        assert s0 == 10.0         # 0*10 + 1*10
        assert scale == 0.5
        assert t == 2.5


def test_flat_allreduce_single_bucket():
    _run(1)


def test_flat_allreduce_bucketed():
    _run(4)
