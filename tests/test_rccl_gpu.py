"""RCCL on one GPU: the first run of the product's collective path under the `nccl`
backend (RCCL on ROCm) -- every other DP test uses gloo.

A world of ONE rank with `BucketedGradAllReduce(force=True)`, which issues its four bucket collectives even
though they are identities at world size 1, so these execute for real:
* RCCL's own stream ordered behind the issuing stream (the weight-gradient stream in the overlapped schedule,
  the compute stream in the serialised one) while the backward still writes the lower layers' gradients;
* `Work.wait()` as a device-side wait of the compute stream before the fused AdamW reads the gradients;
* a step plan's (kdfm/plan.py) replay of the all-reduce's ready() / finish host callbacks.

Check: deterministic mode (ordered reductions), the same three steps -- eager `train_step`, the step a plan
records, one plan replay -- with and without the all-reduce leave BITWISE equal parameters after each step (an
all-reduce of one rank is the identity; a collective that read a gradient before its last write, or an AdamW that
ran before the collective finished, would still be bitwise equal here only by luck of timing, which is why the
race checker models the same ordering: tests/test_race_gpu.py).  Runs in a spawned process: the nccl process group
must not outlive the test.  Reference DP path: Lightning DDP, asr_train_diffm.py:1761-1768.
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


def _steps(eng, batch, ar):
    """eager train_step, the plan-recording step, one plan replay: parameters after each"""
    wav, wl, tg, tl = batch
    out = []
    eng.train_step(wav, wl, tg, tl, ar)
    torch.cuda.synchronize()
    out.append(eng.student.data.detach().clone())
    plan = eng.make_plan(wav, wl, tg, tl, ar)
    torch.cuda.synchronize()
    out.append(eng.student.data.detach().clone())
    plan.replay()
    torch.cuda.synchronize()
    out.append(eng.student.data.detach().clone())
    return out, torch.isfinite(eng.losses).all().item()


def _worker(rank, port, overlapped, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from dataclasses import replace

        from kdfm import kernels as K
        from kdfm.config import DEFAULT
        from kdfm.ddp import BucketedGradAllReduce
        from kdfm.engine import Ver5Engine, synthetic_batch
        cfg = replace(DEFAULT, n_layers=2, deterministic=True)
        K.set_math(cfg.math)
        batch = synthetic_batch(cfg, 4, 32000, 12, dev, seed=77)
        res = {}
        for name, force in (("plain", None), ("rccl", True)):
            eng = Ver5Engine(cfg, dev, teacher_seed=0, student_seed=1, heads_seed=2)
            eng.set_seed(9)
            eng.overlap_wgrad = overlapped   # weight gradients (and the collectives' issue) on the side stream
            ar = None if force is None else BucketedGradAllReduce(eng.student.numel, buckets=4, force=True)
            params, finite = _steps(eng, batch, ar)
            res[name] = (params, finite, None if ar is None else ar.issued)
            del eng
        a, b = res["plain"][0], res["rccl"][0]
        out["backend"] = dist.get_backend()
        out["issued"] = res["rccl"][2]
        out["finite"] = res["plain"][1] and res["rccl"][1]
        out["equal"] = [bool(torch.equal(x, y)) for x, y in zip(a, b)]
        out["maxdiff"] = [float((x - y).abs().max()) for x, y in zip(a, b)]
        out["moved"] = bool(not torch.equal(a[0], a[2]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlapped", [True, False], ids=["overlapped", "serialised"])
def test_rccl_world1_step_equals_no_allreduce(overlapped):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), overlapped, out), nprocs=1, join=True)
    assert out["backend"] == "nccl"
    assert out["finite"]
    assert out["moved"], "the optimizer must change the parameters"
    # 4 buckets per step: the eager step, the recorded step and the replay each issue all four
    assert out["issued"] == 12, out["issued"]
    assert all(out["equal"]), ("parameters differ from the step without the all-reduce", out["maxdiff"])
