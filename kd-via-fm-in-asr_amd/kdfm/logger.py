"""Per-step training metrics as JSON lines, with the reference's metric keys.

The reference logs through Lightning's WandbLogger (asr_train_diffm.py:1744) from training_step
(:814-827): loss/ctc, loss/logit_kd, loss/layer_kd, v/recon, v/kd_pre, v/fm_pre, v/kd_post,
v/fm_post, v/diffkd (use_diffkd only) and train_loss, on_step.  There is no network here, so the same
keys go to a JSONL file, one object per logged step, plus step / lr (and the gradient statistics when
the engine computes them).  Values live on the device: one logged step costs a single
device-to-host copy of a small vector, made on the compute stream after the step's work, so logging
every N steps (Lightning's log_every_n_steps) keeps the other steps free of host synchronisation.
"""
from __future__ import annotations

import json
import os

import torch

_V_KEYS = ("v/recon", "v/kd_pre", "v/fm_pre", "v/kd_post", "v/fm_post")


def step_metrics(eng) -> dict:
    """The reference's training_step log values for the engine's last step, as Python floats.

    Layout read: eng.losses = [total, ctc, logit_kd (already T^2-scaled, before kd_alpha), recon,
    layer KD sum], eng.kd_terms = [recon, kd_pre, fm_pre, kd_post, fm_post, diffkd] (per-layer
    sums, asr_train_diffm.py:773-800), eng.lr, eng.step, eng.grad_stats = [sum g^2, #non-finite].
    kd_model "encfm": asr_train.py's keys (train_ctc_loss, train_logit_kd_loss, train_flow_matching_loss,
    train_router_loss, router/batch_mean_sampling_steps_mean, train_loss) from eng.encfm_stats."""
    encfm = eng.cfg.kd_model == "encfm"
    # the encoder-level FM family (asr_train.py) logs its own key set from eng.encfm_stats = [flow total,
    # router_weight * router total, their sum, mean sampled steps] (:657-663, 770-777)
    terms = eng.encfm_stats if encfm else eng.kd_terms
    parts = [eng.losses, terms, eng.lr, eng.step.to(torch.float32)]
    gs = getattr(eng, "grad_stats", None)
    if gs is not None:
        parts.append(gs)
    with torch.cuda.stream(eng.compute_stream) if eng.losses.is_cuda else _null():
        v = torch.cat([p.reshape(-1).to(torch.float32) for p in parts]).cpu().tolist()
    total, ctc, kl = v[0], v[1], v[2]
    nt = terms.numel()
    t = v[5:5 + nt]
    if eng.cfg.kd_model == "logitkd":
        # DistilEncDecCTCModelBPE.training_step (asr_train_diffm.py:282, 318-320)
        out = {"train_kd_loss": kl, "train_ctc_loss": ctc}
    elif encfm:
        out = {"train_ctc_loss": ctc, "train_logit_kd_loss": kl, "train_flow_matching_loss": t[0]}
        if eng.cfg.encfm_dynamic:
            out["train_router_loss"] = t[1]
            out["router/batch_mean_sampling_steps_mean"] = t[3]
    else:
        out = {"loss/ctc": ctc, "loss/logit_kd": kl, "loss/layer_kd": 0.0}
        for k, x in zip(_V_KEYS, t[:5]):
            out[k] = x
        if eng.cfg.use_diffkd:
            out["v/diffkd"] = t[5]
    out["train_loss"] = total
    out["lr"] = v[5 + nt]
    out["step"] = int(v[6 + nt])
    if gs is not None:
        out["grad_norm"] = v[7 + nt] ** 0.5
        out["grad_nonfinite"] = int(v[8 + nt])
    return out


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class JsonlLogger:
    """Append step_metrics(eng) to `path` every `every` steps (rank 0 only in multi-process runs)."""

    def __init__(self, path: str, every: int = 1, rank: int = 0):
        self.path = path
        self.every = max(1, int(every))
        self.rank = rank
        self._n = 0
        self._fh = None
        if rank == 0:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def __call__(self, eng, **extra):
        """Call once per training step, after it was issued; returns the metrics when logged."""
        self._n += 1
        if self._fh is None or (self._n - 1) % self.every:
            return None
        m = step_metrics(eng)
        m.update(extra)
        self._fh.write(json.dumps(m, sort_keys=False) + "\n")
        return m

    def close(self):
        if self._fh is not None:
            self._fh.close()
            self._fh = None


def read_jsonl(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


__all__ = ["JsonlLogger", "step_metrics", "read_jsonl"]
