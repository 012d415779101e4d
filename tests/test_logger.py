"""kdfm.logger: the reference's training_step log keys (asr_train_diffm.py:814-827) as JSON lines."""
import json
import types

import torch

from kdfm.logger import JsonlLogger, read_jsonl, step_metrics

REF_KEYS = ["loss/ctc", "loss/logit_kd", "loss/layer_kd", "v/recon", "v/kd_pre", "v/fm_pre", "v/kd_post", "v/fm_post",
            "train_loss"]


def _fake_engine(diffkd=False, grad=False):
    # the engine's device buffers, on the CPU here: losses [total, ctc, kl, recon, layer KD],
    # kd_terms [recon, kd_pre, fm_pre, kd_post, fm_post, diffkd]
    return types.SimpleNamespace(
        cfg=types.SimpleNamespace(use_diffkd=diffkd, kd_model="diffm"),
        losses=torch.tensor([10.0, 6.0, 1.5, 0.25, 2.0]),
        kd_terms=torch.tensor([0.25, 0.0, 0.0, 0.0, 1.75, 0.5]),
        lr=torch.tensor([1e-3]), step=torch.tensor([7], dtype=torch.int64),
        grad_stats=torch.tensor([16.0, 0.0]) if grad else None, compute_stream=None)


def test_step_metrics_keys_and_values():
    m = step_metrics(_fake_engine())
    assert list(m)[:len(REF_KEYS)] == REF_KEYS
    assert m["loss/ctc"] == 6.0 and m["loss/logit_kd"] == 1.5 and m["train_loss"] == 10.0
    assert m["v/recon"] == 0.25 and m["v/fm_post"] == 1.75 and m["v/kd_pre"] == 0.0
    assert "v/diffkd" not in m and m["step"] == 7 and abs(m["lr"] - 1e-3) < 1e-9
    m = step_metrics(_fake_engine(diffkd=True, grad=True))
    assert m["v/diffkd"] == 0.5 and m["grad_norm"] == 4.0 and m["grad_nonfinite"] == 0


def test_step_metrics_encfm_keys():
    """kd_model 'encfm' (asr_train.py): train_ctc_loss, train_logit_kd_loss, train_flow_matching_loss,
    train_router_loss (router_weight-scaled), router/batch_mean_sampling_steps_mean, train_loss
    (:657-663, 770-777) from eng.encfm_stats = [flow, weighted router, sum, mean steps]; no v/* keys."""
    eng = _fake_engine()
    eng.cfg = types.SimpleNamespace(use_diffkd=False, kd_model="encfm", encfm_dynamic=True)
    eng.encfm_stats = torch.tensor([3.0, 0.5, 3.5, 4.25])
    m = step_metrics(eng)
    assert list(m)[:6] == ["train_ctc_loss", "train_logit_kd_loss", "train_flow_matching_loss", "train_router_loss",
                           "router/batch_mean_sampling_steps_mean", "train_loss"]
    assert m["train_flow_matching_loss"] == 3.0 and m["train_router_loss"] == 0.5
    assert m["router/batch_mean_sampling_steps_mean"] == 4.25 and m["train_loss"] == 10.0
    assert not any(k.startswith("v/") for k in m) and m["step"] == 7 and abs(m["lr"] - 1e-3) < 1e-9
    eng.cfg.encfm_dynamic = False
    m = step_metrics(eng)
    assert "train_router_loss" not in m and m["train_flow_matching_loss"] == 3.0


def test_jsonl_logger_every_n(tmp_path):
    path = str(tmp_path / "logs" / "train.jsonl")
    log = JsonlLogger(path, every=3)
    eng = _fake_engine()
    got = [log(eng, epoch=0) for _ in range(7)]
    log.close()
    assert [g is not None for g in got] == [True, False, False, True, False, False, True]
    rows = read_jsonl(path)
    assert len(rows) == 3 and all(set(REF_KEYS) <= set(r) for r in rows) and rows[0]["epoch"] == 0
    with open(path) as f:
        assert all(json.loads(line)["train_loss"] == 10.0 for line in f)


def test_jsonl_logger_non_zero_rank_writes_nothing(tmp_path):
    path = str(tmp_path / "r1.jsonl")
    log = JsonlLogger(path, rank=1)
    assert log(_fake_engine()) is None
    log.close()
    import os
    assert not os.path.exists(path)
