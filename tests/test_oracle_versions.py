"""Oracle for KD versions 1-8 (oracle/ver5.py:v_layer_losses) against golden vectors generated
from the reference's own `_compute_v_losses_one_layer` (tests/golden/make_golden_versions.py,
asr_train_diffm.py:645-729): the five loss terms, d(total)/d(s), per-parameter gradient checksums."""
import os

import numpy as np
import pytest
import torch

from oracle import ver5 as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_heads_versions.npz")
KEYS = ("recon_loss", "kd_loss_pre", "fm_loss_pre", "kd_loss_post", "fm_loss_post")
CASES = [(v, "mse") for v in range(1, 9)] + [(1, "l1"), (3, "l1"), (8, "l1")]


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def params(gold):
    return {k[len("param."):]: torch.tensor(v, requires_grad=True) for k, v in gold.items() if k.startswith("param.")}


@pytest.mark.parametrize("version,kd", CASES)
def test_oracle_versions_match_reference(gold, version, kd):
    p = params(gold)
    s = torch.tensor(gold["in.s"], requires_grad=True)
    out = O.v_layer_losses(version, s, torch.tensor(gold["in.t"]), p, torch.tensor(gold["in.eps"]), kd=kd)
    tag = f"v{version}{kd}"
    for k in KEYS:
        np.testing.assert_allclose(float(out[k]), float(gold[f"{tag}.{k}"]), rtol=1e-5, atol=1e-7, err_msg=k)
    total = sum(out[k] for k in KEYS)
    names = list(p)
    grads = torch.autograd.grad(total, [p[n] for n in names] + [s], allow_unused=True)
    np.testing.assert_allclose(grads[-1].numpy(), gold[f"{tag}.grad.s"], rtol=1e-4, atol=1e-7)
    for n, g in zip(names, grads[:-1]):
        g = torch.zeros_like(p[n]) if g is None else g
        ref = gold[f"{tag}.gsum.{n}"]
        got = np.array([float(g.double().sum()), float((g.double() ** 2).sum())])
        np.testing.assert_allclose(got, ref, rtol=2e-4, atol=1e-9, err_msg=n)
