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


def _worker_overlap(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kd-via-fm-in-asr_amd"))
    from kdfm.config import DEFAULT, student_specs
    from kdfm.ddp import BucketedGradAllReduce
    from kdfm.store import FlatStore
    st = FlatStore(student_specs(DEFAULT), "cpu", with_grad=True)
    n = st.numel
    ar = BucketedGradAllReduce(n, buckets=4)
    gen = torch.Generator().manual_seed(100 + rank)
    st.grad.copy_(torch.randn(n, generator=gen))
    ref = st.grad.clone()
    # the engine's readiness order: heads, decoder, layers 15..0 (each a flat suffix), then the rest
    off = st.offsets
    launched = []
    heads0 = min(o for k, o in off.items() if not k.startswith(("encoder.", "decoder.")))
    ar.ready(st.grad, heads0)
    launched.append(len(ar._launched))
    ar.ready(st.grad, off["decoder.decoder_layers.0.weight"])
    for i in range(DEFAULT.n_layers - 1, -1, -1):
        ar.ready(st.grad, min(o for k, o in off.items() if k.startswith(f"encoder.layers.{i}.")))
        launched.append(len(ar._launched))
    scale = ar(st.grad)
    allref = [torch.empty_like(ref) for _ in range(world)]
    dist.all_gather(allref, ref)
    exp = allref[0] + allref[1]
    out[rank] = (float((st.grad - exp).abs().max()), scale, launched, ar.edges)
    dist.destroy_process_group()


def test_bucketed_overlap_ready_order():
    """BucketedGradAllReduce with the engine's ready() sequence (reverse layer order) sums every
    bucket exactly once, launches buckets before the backward ends, and leaves the last for __call__."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_overlap, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        err, scale, launched, edges = out[r]
        assert err == 0.0
        assert scale == 0.5
        assert len(edges) == 5 and edges[0] == 0
        assert launched[-1] >= 3          # >= 3 of 4 buckets in flight before the subsampling grads
        assert launched == sorted(launched)
