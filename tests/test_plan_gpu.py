"""Step plans (kdfm/plan.py, Ver5Engine.make_plan): one recorded training step replayed without the
Python wrappers must BE the step.  Two engines start from the same weights and seeds; one runs eager
train_step, the other records a plan (the recording itself is a real step) and replays it.  With
ordered reductions (deterministic=True) and the benchmark's overlapped weight-gradient stream, every
parameter, AdamW moment and BatchNorm running statistic must be bitwise equal after 4 steps (the
losses to 1e-5: their scalar accumulators use float atomics),
and the replay must issue exactly the recorded launches (cut the host issue)."""
from dataclasses import replace

import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(cfg):
    from kdfm.engine import Ver5Engine
    eng = Ver5Engine(cfg, "cuda", teacher_seed=0, student_seed=1, heads_seed=2)
    eng.overlap_wgrad = True
    eng.set_seed(91)
    return eng


def test_plan_replay_equals_eager_steps():
    from kdfm.config import DEFAULT
    from kdfm.engine import synthetic_batch
    cfg = replace(DEFAULT, n_layers=4, deterministic=True)
    wav, wl, tg, tl = synthetic_batch(cfg, 4, 64000, 30, "cuda", seed=5)
    a, b = _engine(cfg), _engine(cfg)
    a.train_step(wav, wl, tg, tl)       # warm-up step on both: lazily created workspaces
    b.train_step(wav, wl, tg, tl)
    plan = b.make_plan(wav, wl, tg, tl)   # the recording is step 2 of b
    a.train_step(wav, wl, tg, tl)         # step 2 of a
    assert len(plan) > 100
    for _ in range(2):
        a.train_step(wav, wl, tg, tl)
        plan.replay()
    torch.cuda.synchronize()
    # scalar loss accumulators keep float atomics (deterministic mode orders every reduction that feeds
    # a gradient, not the loss sums): 1e-5 relative, like tests/test_determinism_gpu.py
    torch.testing.assert_close(a.losses, b.losses, rtol=1e-5, atol=0.0)
    for name in ("data", "exp_avg", "exp_avg_sq"):
        x, y = getattr(a.student, name), getattr(b.student, name)
        assert torch.equal(x, y), f"student.{name} differs: {(x - y).abs().max().item():.3e}"
    assert torch.equal(a.bn.data, b.bn.data)
    assert int(a.step) == int(b.step) == 4


def test_plan_rejects_unreplayable_torch_ops():
    from kdfm.plan import PlanError, StepPlan
    x = torch.zeros(16, device="cuda")
    with pytest.raises(PlanError):
        StepPlan().record(lambda: x.add_(1.0))
