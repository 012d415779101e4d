"""oracle/encfm.py (encoder-level flow matching + DynamicStepRouter, asr_train.py:595-666, 1021-1377)
against tests/golden/kd_encfm.npz, made from the reference's own classes (make_golden_encfm.py):
per-layer router steps and chosen S exactly, losses rtol 1e-5, FM output and every gradient (all
parameters and every hooked student layer) max|diff| <= 1e-5 * max|ref| + 1e-7, for all four step
strategies."""
import os

import numpy as np
import pytest
import torch

from oracle import encfm as E

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_encfm.npz")


@pytest.mark.parametrize("strategy", E.STRATEGIES)
def test_encfm_oracle_matches_reference(strategy):
    z = dict(np.load(GOLD, allow_pickle=False))
    L = int(z["meta.L"])
    P = {k[6:]: torch.tensor(v).requires_grad_(True) for k, v in z.items() if k.startswith("param.")}
    s = [torch.tensor(z[f"in.s{i}"]).requires_grad_(True) for i in range(L)]
    t = [torch.tensor(z[f"in.t{i}"]) for i in range(L)]
    g = [torch.tensor(z[f"in.gumbel{i}"]) for i in range(L)]
    R = torch.tensor(z["in.R"])
    out = E.encfm_forward(P, s, t, g, strategy=strategy)
    pre = strategy + "."
    assert torch.equal(out["steps"], torch.tensor(z[pre + "steps"]))
    assert out["S"] == z[pre + "S"].tolist()
    np.testing.assert_allclose(float(out["total"].detach()), float(z[pre + "total"]), rtol=1e-5)
    np.testing.assert_allclose([float(x) for x in out["flow"]], z[pre + "flow"], rtol=1e-5)
    np.testing.assert_allclose([float(x) for x in out["router_loss"]], z[pre + "router_loss"], rtol=1e-5, atol=1e-7)

    def close(a, b, what):
        a = a.detach().double().numpy()
        err = np.abs(a - b).max()
        assert err <= 1e-5 * np.abs(b).max() + 1e-7, f"{what}: {err:.3e} vs max {np.abs(b).max():.3e}"

    close(out["fm_out"], z[pre + "fm_out"], "fm_out")
    obj = out["total"] + (out["fm_out"] * R).sum()
    names = list(P)
    grads = torch.autograd.grad(obj, [P[n] for n in names] + s, allow_unused=True)
    for n, gr in zip(names, grads[:len(names)]):
        close(torch.zeros_like(P[n]) if gr is None else gr, z[pre + "grad." + n], "grad " + n)
    for i in range(L):
        close(grads[len(names) + i], z[pre + f"grad.s{i}"], f"grad s{i}")


def test_choose_steps_tie_rules():
    st = torch.tensor([3, 5, 5, 3, 1, 2])
    assert E.choose_steps(st, "batch_mode", 8) == 3          # smallest of the tied modes
    assert E.choose_steps(torch.tensor([1, 2, 3, 4]), "batch_median", 8) == 2   # lower median
    assert E.choose_steps(torch.tensor([1, 2, 2, 4]), "batch_avg", 8) == 2      # round(2.25)
    assert E.choose_steps(torch.tensor([1, 2, 3, 4]), "batch_avg", 8) == 2      # round half to even (2.5)


def test_schedule_coeffs():
    assert E.schedule_coeffs(4, "rectified") == (1.0, -1.0)
    ca, cv = E.schedule_coeffs(8, "vp_ode")
    assert np.isfinite(ca) and np.isfinite(cv) and cv < 0
    with pytest.raises(ValueError):
        E.schedule_coeffs(8, "ve_ode")
