"""Bucketed, backward-overlapped gradient all-reduce (kdfm/ddp.py BucketedGradAllReduce) driven by
the real engine backward on the GPU: two ranks share cuda:0 over gloo (RCCL needs one GPU per rank;
the 1-GPU box cannot host an nccl world of 2), so this checks the stream ordering of the overlap -
the comm stream waits for the main stream and the weight-gradient side stream before each bucket -
against a plain all-reduce of the finished local gradients.  The engine runs in its default
(non-deterministic, overlapped weight-gradient stream) mode, whose repeated runs differ by float
summation order; the tolerance is the larger of 1e-4 x max|grad| and 8x the run-to-run difference
measured here — a mis-ordered bucket would be off by O(|grad|) over whole buckets."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
    from dataclasses import replace

    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.ddp import BucketedGradAllReduce
    from kdfm.engine import Ver5Engine, synthetic_batch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = replace(DEFAULT, n_layers=3)
    K.set_math(cfg.math)
    eng = Ver5Engine(cfg, dev)
    eng.set_seed(77 + rank)
    wav, wl, tg, tl = synthetic_batch(cfg, 4, 48000, 20, dev, seed=300 + rank)
    eng.advance_rng()
    ctx = eng.forward(wav, wl, tg, tl, train=True)
    eng.backward(ctx)
    del ctx
    torch.cuda.synchronize()
    ref = eng.student.grad.clone()
    ctx = eng.forward(wav, wl, tg, tl, train=True)   # same RNG state: run-to-run float noise only
    eng.backward(ctx)
    del ctx
    torch.cuda.synchronize()
    noise = float((eng.student.grad - ref).abs().max())
    dist.all_reduce(ref)
    ar = BucketedGradAllReduce(eng.student.numel, buckets=4)
    grad = eng.student.grad
    ctx = eng.forward(wav, wl, tg, tl, train=True)   # same RNG state: same masks as above
    eng.backward(ctx, grad_ready=lambda o: ar.ready(grad, o))
    early = len(ar._launched)
    del ctx
    scale = ar(grad)
    torch.cuda.synchronize()
    tol = max(1e-4 * ref.abs().max().item(), 8.0 * noise)
    out[rank] = (float((grad - ref).abs().max()), tol, scale, early)
    dist.destroy_process_group()


def test_bucketed_overlap_matches_flat_allreduce():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        err, tol, scale, early = out[r]
        assert err <= tol, (err, tol)
        assert scale == 0.5
        assert early >= 3    # buckets launched while the backward was still running
