"""The CPU oracle's DiffKD head (oracle/ver5.py diffkd) against golden vectors generated from the
reference's own DiffKDModule (tests/golden/make_golden_diffkd.py, asr_train_diffm.py:326-394 and the
training_step mean over layer pairs :795-800): loss, d(loss)/d(student layer outputs) and every
parameter gradient (float64 evaluation of the restatement, float32 fixtures: 1e-5 relative)."""
import os

import numpy as np
import torch

from oracle import ver5 as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kd_diffkd.npz")


def test_diffkd_matches_reference_fixture():
    z = np.load(GOLD)
    L, steps = int(z["meta.L"]), int(z["meta.steps"])
    p = {k[6:]: torch.tensor(z[k], dtype=torch.float64) for k in z.files if k.startswith("param.")}
    p = {"diffkd." + k: v.requires_grad_(True) for k, v in p.items()}
    s = [torch.tensor(z[f"in.s{i}"], dtype=torch.float64).requires_grad_(True) for i in range(L)]
    t = [torch.tensor(z[f"in.t{i}"], dtype=torch.float64) for i in range(L)]
    loss = sum(O.diffkd(si, ti, p, steps) for si, ti in zip(s, t)) / L
    assert abs(loss.item() - float(z["loss"])) <= 1e-5 * abs(float(z["loss"]))
    names = list(p)
    grads = torch.autograd.grad(loss, [p[n] for n in names] + s, allow_unused=True)
    for n, g in zip(names, grads[:len(names)]):
        key = "grad." + n[len("diffkd."):]
        if key not in z.files:   # the encoder: no gradient in the reference
            assert g is None, n
            continue
        ref = torch.tensor(z[key], dtype=torch.float64)
        assert (g - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-9, n
    for i in range(L):
        ref = torch.tensor(z[f"grad.s{i}"], dtype=torch.float64)
        assert (grads[len(names) + i] - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-9


def test_diffkd_trainable_set():
    cfg = O.StepConfig(n_layers=2)
    p = O.init_all(cfg)
    names = O.trainable_names(p, 5, use_diffkd=True)
    assert "diffkd.decoder.weight" in names and "diffkd.denoiser.2.bias" in names
    assert not any(n.startswith("diffkd.encoder.") for n in names)
    assert not any(n.startswith("diffkd.") for n in O.trainable_names(p, 5))
