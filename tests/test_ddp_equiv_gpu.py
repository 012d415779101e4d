"""Data-parallel gradient equivalence on the GPU engine.

Two ranks (world size 2, gloo over CUDA tensors, both on cuda:0 — the box has one GPU; the product
runs RCCL, the bucketing/overlap logic under test is the same) each run the f32 deterministic
engine (PARITY) on their own shard of one batch, with kdfm.ddp.BucketedGradAllReduce hooked into the
backward exactly as Ver5Engine.train_step does (4 buckets launched in reverse layer order while the
backward continues).  Each rank also runs BOTH shards single-process, with no collective.

Checks (bitwise — deterministic mode makes every shard gradient reproducible, and a two-term f32
sum is order-free):
* the all-reduced flat gradient equals G(shard 0) + G(shard 1) on both ranks;
* after the fused AdamW step with the returned 1/world scale, both ranks hold identical parameters,
  equal to a single-process AdamW step on the mean gradient.
BatchNorm statistics stay per rank (as in the reference, no sync_batchnorm), which is why the
comparison is against per-shard gradients and not a single B=4 batch.
"""
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


def _batch(cfg):
    g = torch.Generator().manual_seed(5)
    B, N, U = 4, 24000, 9
    wav = 0.1 * torch.randn(B, N, generator=g)
    wl = torch.tensor([24000, 19000, 24000, 15500], dtype=torch.int64)
    tg = torch.randint(0, cfg.vocab, (B, U), generator=g)
    tl = torch.tensor([9, 7, 8, 6], dtype=torch.int64)
    T = ((N // cfg.hop) // 2) // 2 + 1
    eps = torch.randn(cfg.n_layers, B, T, cfg.latent, generator=g)
    return wav, wl, tg, tl, eps


def _shard(batch, s, dev):
    wav, wl, tg, tl, eps = batch
    sl = slice(2 * s, 2 * s + 2)
    L, _, T, D = eps.shape
    return (wav[sl].to(dev), wl[sl].to(dev), tg[sl].to(dev), tl[sl].to(dev),
            eps[:, sl].reshape(L * 2 * T, D).contiguous().to(dev))


def _engine(cfg, dev):
    from kdfm.engine import Ver5Engine
    eng = Ver5Engine(cfg, dev, teacher_seed=0, student_seed=1, heads_seed=2)
    eng.set_seed(3)
    return eng


def _grad(eng, sh, ready=None):
    wav, wl, tg, tl, eps = sh
    ctx = eng.forward(wav, wl, tg, tl, train=True, eps=eps)
    grad = eng.student.grad
    eng.backward(ctx, grad_ready=(lambda o: ready(grad, o)) if ready is not None else None)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kdfm.config import PARITY
        from kdfm.ddp import BucketedGradAllReduce
        cfg = PARITY
        dev = torch.device("cuda:0")
        batch = _batch(cfg)
        eng = _engine(cfg, dev)
        local = []
        for s in range(world):
            _grad(eng, _shard(batch, s, dev))
            torch.cuda.synchronize()
            local.append(eng.student.grad.clone())
        ar = BucketedGradAllReduce(eng.student.numel, buckets=4)
        _grad(eng, _shard(batch, rank, dev), ready=ar.ready)
        launched_early = len(ar._launched)
        scale = eng.allreduce_grads(ar)   # as Ver5Engine.train_step: on the engine's compute stream
        torch.cuda.synchronize()
        g_sum = local[0] + local[1]
        g_ddp = eng.student.grad.clone()
        eng.optimizer_step(scale)
        # single-process reference step on the mean gradient
        ref = _engine(cfg, dev)
        ref.student.grad.copy_(g_sum)
        ref.optimizer_step(0.5)
        torch.cuda.synchronize()
        p = eng.student.data.detach().cpu()
        both = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(both, p)
        diff = (g_ddp - g_sum).abs()
        worst = int(diff.argmax())
        where = max(((o, k) for k, o in eng.student.offsets.items() if o <= worst), default=(0, "?"))[1]
        out[rank] = dict(
            grad_equal=bool(torch.equal(g_ddp, g_sum)),
            grad_maxdiff=float(diff.max()),
            grad_where=(where, worst, int((diff > 0).sum()), float(g_sum.abs()[worst]),
                        float(local[0].abs()[worst]), float(local[1].abs()[worst]), float(g_ddp[worst])),
            shard_differs=bool(not torch.equal(local[0], local[1])),
            scale=scale, launched_early=launched_early,
            ranks_equal=bool(torch.equal(both[0], both[1])),
            ref_equal=bool(torch.equal(p, ref.student.data.detach().cpu())),
            finite=bool(torch.isfinite(g_ddp).all()))
    finally:
        dist.destroy_process_group()


def test_ddp_gradients_equal_sum_of_shard_gradients():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        o = out[r]
        assert o["finite"]
        assert o["shard_differs"], "the two shards must give different gradients"
        assert o["grad_equal"], (r, o["grad_maxdiff"], o["grad_where"])
        assert o["scale"] == 0.5
        assert o["launched_early"] >= 3, "buckets must be launched while the backward runs"
        assert o["ranks_equal"], "parameters diverged across ranks after the AdamW step"
        assert o["ref_equal"], "DDP step differs from a single-process step on the mean gradient"
