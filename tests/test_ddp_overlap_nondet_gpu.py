"""The benchmark's production DDP mode -- weight gradients on the overlapped side stream, atomic
(non-deterministic) reductions, 4 buckets launched from inside the backward -- checked WITHOUT needing
run-to-run determinism: at every bucket launch the bucket is snapshotted
on the issuing stream, i.e. exactly what the collective reads.

* collective run: after the step the reduced bucket must equal the sum of both ranks' snapshots BITWISE
  (a two-term f32 sum is order-free), so nothing wrote the bucket between the launch and the end of the
  step, and the collective read what the snapshot saw;
* snapshot-only run (no collective): the snapshot must equal the finished local gradient BITWISE, so
  every gradient of the bucket was final when it launched (no backward work after the launch point).

Two gloo ranks share cuda:0 (the 1-GPU box cannot host an RCCL world of 2; the ordering under test --
the issuing stream after the compute and weight-gradient streams -- is the same)."""
import os
import socket
import sys

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
    sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dataclasses import replace

        from kdfm import kernels as K
        from kdfm.config import DEFAULT
        from kdfm.ddp import BucketedGradAllReduce
        from kdfm.engine import Ver5Engine, synthetic_batch

        class Snapshot(BucketedGradAllReduce):
            def __init__(self, numel, collective):
                super().__init__(numel, buckets=4)
                self.collective = collective
                self.snaps = {}

            def _issue(self, chunk, k):
                self.snaps[k] = chunk.clone()   # on the issuing stream, where the collective reads
                return super()._issue(chunk, k) if self.collective else None

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cfg = replace(DEFAULT, n_layers=4, deterministic=False)
        K.set_math(cfg.math)
        eng = Ver5Engine(cfg, dev)
        assert not eng._serial(), "the benchmark's overlapped schedule"
        eng.set_seed(91 + rank)
        wav, wl, tg, tl = synthetic_batch(cfg, 4, 64000, 24, dev, seed=500 + rank)
        grad = eng.student.grad
        res = {}
        for collective in (False, True):
            ar = Snapshot(eng.student.numel, collective)
            eng.advance_rng()
            ctx = eng.forward(wav, wl, tg, tl, train=True)
            eng.backward(ctx, grad_ready=lambda o: ar.ready(grad, o))
            early = len(ar._launched)
            del ctx
            scale = eng.allreduce_grads(ar)   # as Ver5Engine.train_step: on the engine's compute stream
            torch.cuda.synchronize()
            bad = []
            for k, snap in sorted(ar.snaps.items()):
                lo, hi = ar.edges[k], ar.edges[k + 1]
                if collective:
                    peers = [torch.empty_like(snap) for _ in range(world)]
                    dist.all_gather(peers, snap)
                    want = peers[0] + peers[1]
                else:
                    want = snap
                d = (grad[lo:hi] - want).abs()
                if not torch.equal(grad[lo:hi], want):
                    i = int(d.argmax()) + lo
                    name = max(((o, n) for n, o in eng.student.offsets.items() if o <= i), default=(0, "?"))[1]
                    bad.append((k, float(d.max()), int((d > 0).sum()), name))
            res[collective] = dict(bad=bad, early=early, scale=scale, n=len(ar.snaps),
                                   finite=bool(torch.isfinite(grad).all()))
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_overlapped_nondeterministic_buckets_reduce_their_launch_snapshots():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        for collective, o in out[r].items():
            what = "reduced bucket != sum of launch snapshots" if collective else "launch snapshot != final gradient"
            assert not o["bad"], f"rank {r}: {what}: (bucket, max diff, #elements, first param) {o['bad']}"
            assert o["n"] == 4 and o["early"] >= 3 and o["finite"]
            assert o["scale"] == 0.5
