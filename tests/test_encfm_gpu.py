"""Encoder-level flow matching + DynamicStepRouter on the engine (kdfm/encfm.py, csrc/encfm.hip)
against (a) tests/golden/kd_encfm.npz, made from the REFERENCE'S OWN DynamicStepRouter and
FlowMatchingModule (make_golden_encfm.py; asr_train.py:595-666, 1021-1377), for all four step
strategies with the recorded Gumbel noise injected, and (b) oracle/encfm.py in float64 at a size that
takes the kernels' multi-tile paths (3 layers x 5 utterances x 203 frames, ragged group sizes).

Exact: the router's sampled steps and every segment's flow step count.  Router losses and router
gradients (f32 VALU kernels and f32 weight gradients): rtol 1e-4.  The FM chain runs bf16 MFMA with f32
state: flow losses rtol 2e-2, the last layer's FM output and every FM / feature gradient relative
Frobenius <= 3e-2 (the tolerances of the other fused bf16 chains)."""
import os
from dataclasses import replace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "kd_encfm.npz")


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _cfg(L, strategy, **kw):
    from kdfm.config import DEFAULT
    args = dict(n_layers=L, kd_model="encfm", encfm_strategy=strategy, encfm_dynamic=True, router_max_steps=8)
    args.update(kw)
    return replace(DEFAULT, **args)


def _run(cfg, P, s, t, gumbel, B, T, R):
    """forward + backward of the encfm block alone; returns (ws, dfeats, G)."""
    from kdfm import kernels as K
    from kdfm.encfm import EncFMWorkspace, encfm_backward, encfm_forward, encfm_specs
    dev = torch.device("cuda")
    L = cfg.n_layers
    ws = EncFMWorkspace(cfg, B, T, dev)
    G = {n: torch.zeros(shape, device=dev) for n, shape in encfm_specs(cfg)}
    with K.mode("bf16", True):
        encfm_forward(cfg, P, s, t, ws, train=True, gumbel=gumbel)
        dfeats = torch.empty(L * B * T, cfg.d_student, device=dev)
        encfm_backward(cfg, P, G, ws, dfeats, R, lambda fn, *keep: fn())
    torch.cuda.synchronize()
    return ws, dfeats, G


@pytest.mark.parametrize("strategy", ["batch_mode", "batch_avg", "batch_median", "group"])
def test_encfm_matches_reference(strategy):
    z = dict(np.load(GOLD, allow_pickle=False))
    L, B, T = int(z["meta.L"]), int(z["meta.B"]), int(z["meta.T"])
    dev = torch.device("cuda")
    cfg = _cfg(L, strategy)
    P = {k[6:]: torch.tensor(v).to(dev).contiguous() for k, v in z.items() if k.startswith("param.")}
    s = torch.stack([torch.tensor(z[f"in.s{i}"]).reshape(B * T, -1) for i in range(L)]).to(dev).contiguous()
    t = torch.stack([torch.tensor(z[f"in.t{i}"]).reshape(B * T, -1) for i in range(L)]).to(dev).contiguous()
    g = torch.cat([torch.tensor(z[f"in.gumbel{i}"]) for i in range(L)]).to(dev).contiguous()
    R = torch.tensor(z["in.R"]).reshape(B * T, -1).to(dev).contiguous()
    ws, dfeats, G = _run(cfg, P, s, t, g, B, T, R)
    pre = strategy + "."
    steps = z[pre + "steps"]
    assert np.array_equal(ws.steps.cpu().numpy().reshape(L, B), steps)
    S = ws.S.cpu().numpy().reshape(L, B)
    for i in range(L):
        want = steps[i] if strategy == "group" else np.full(B, z[pre + "S"][i])
        assert np.array_equal(S[i], want), (i, S[i], want)
    np.testing.assert_allclose(ws.rloss.cpu().numpy(), z[pre + "router_loss"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(ws.flow.cpu().numpy(), z[pre + "flow"], rtol=2e-2)
    np.testing.assert_allclose(ws.stats[2].item(), float(z[pre + "total"]), rtol=2e-2)
    assert _rel(ws.xS.view(B, T, -1), z[pre + "fm_out"]) <= 3e-2
    d = dfeats.view(L, B, T, -1)
    for i in range(L):
        assert _rel(d[i], z[pre + f"grad.s{i}"]) <= 3e-2, f"d/ds layer {i}: {_rel(d[i], z[pre + f'grad.s{i}'])}"
    for n, gr in G.items():
        ref = z[pre + "grad." + n]
        tol = 1e-4 if n.startswith("router.") else 3e-2
        if np.abs(ref).max() == 0.0:
            assert gr.abs().max().item() == 0.0, n
            continue
        assert _rel(gr, ref) <= tol, f"grad {n}: {_rel(gr, ref):.3e}"


def test_encfm_matches_oracle_multitile():
    """3 layers x 5 utterances x 203 frames (3045 rows: many 32-row tiles, partial last tile, tiles
    straddling utterances and layers), group strategy (ragged per-utterance step counts) vs the float64
    oracle with the same Gumbel noise; and determinism (two runs bitwise equal apart from the float-atomic
    per-layer loss sums)."""
    from oracle import encfm as E
    L, B, T = 3, 5, 203
    dev = torch.device("cuda")
    cfg = _cfg(L, "group")
    P64 = E.init_encfm(L=L, seed=3)
    P64 = {k: v.double() for k, v in P64.items()}
    g = torch.Generator().manual_seed(9)
    s = [0.5 * torch.randn(B, T, 88, generator=g, dtype=torch.float64) for _ in range(L)]
    t = [torch.randn(B, T, 176, generator=g, dtype=torch.float64) for _ in range(L)]
    gum = [-torch.empty(B, 8, dtype=torch.float64).exponential_(generator=g).log() for _ in range(L)]
    R = torch.randn(B, T, 88, generator=g, dtype=torch.float64)
    for p in P64.values():
        p.requires_grad_(True)
    sg = [x.clone().requires_grad_(True) for x in s]
    out = E.encfm_forward(P64, sg, t, gum, strategy="group")
    obj = out["total"] + (out["fm_out"] * R).sum()
    names = list(P64)
    grads = torch.autograd.grad(obj, [P64[n] for n in names] + sg, allow_unused=True)
    P = {k: v.detach().float().to(dev).contiguous() for k, v in P64.items()}
    sd = torch.stack([x.reshape(B * T, -1) for x in s]).float().to(dev).contiguous()
    td = torch.stack([x.reshape(B * T, -1) for x in t]).float().to(dev).contiguous()
    gd = torch.cat(gum).float().to(dev).contiguous()
    Rd = R.reshape(B * T, -1).float().to(dev).contiguous()
    ws, dfeats, G = _run(cfg, P, sd, td, gd, B, T, Rd)
    assert torch.equal(ws.steps.cpu().view(L, B).long(), out["steps"])
    assert torch.equal(ws.S.cpu().view(L, B).long(), out["steps"])
    np.testing.assert_allclose(ws.flow.cpu().numpy(), [float(x) for x in out["flow"]], rtol=2e-2)
    np.testing.assert_allclose(ws.rloss.cpu().numpy(), [float(x) for x in out["router_loss"]], rtol=1e-4, atol=1e-7)
    assert _rel(ws.xS.view(B, T, -1), out["fm_out"].detach()) <= 3e-2
    d = dfeats.view(L, B, T, -1)
    for i in range(L):
        assert _rel(d[i], grads[len(names) + i]) <= 3e-2, i
    for n, gr in zip(names, grads[:len(names)]):
        ref = torch.zeros_like(P64[n]) if gr is None else gr
        tol = 1e-4 if n.startswith("router.") else 3e-2
        assert _rel(G[n], ref) <= tol, f"grad {n}: {_rel(G[n], ref):.3e}"
    ws2, d2, G2 = _run(cfg, P, sd, td, gd, B, T, Rd)
    assert torch.equal(dfeats, d2) and torch.equal(ws.xS, ws2.xS)
    for n in G:
        assert torch.equal(G[n], G2[n]), n


def test_encfm_fixed_steps():
    """use_dynamic_steps=False with sampling_steps_per_layer: no router, each layer's fixed S."""
    from oracle import encfm as E
    L, B, T = 2, 3, 50
    dev = torch.device("cuda")
    cfg = _cfg(L, "batch_mode", encfm_dynamic=False, encfm_steps_per_layer=(3, 6))
    P64 = {k: v.double() for k, v in E.init_encfm(L=L, seed=5).items() if k.startswith("flow_matching.")}
    g = torch.Generator().manual_seed(2)
    s = [0.5 * torch.randn(B, T, 88, generator=g, dtype=torch.float64) for _ in range(L)]
    t = [torch.randn(B, T, 176, generator=g, dtype=torch.float64) for _ in range(L)]
    flows = [E.fm_forward(P64, s[i], t[i], S)[0].item() for i, S in enumerate((3, 6))]
    _, xS = E.fm_forward(P64, s[1], t[1], 6)
    P = {k: v.float().to(dev).contiguous() for k, v in P64.items()}
    sd = torch.stack([x.reshape(B * T, -1) for x in s]).float().to(dev).contiguous()
    td = torch.stack([x.reshape(B * T, -1) for x in t]).float().to(dev).contiguous()
    ws, _, _ = _run(cfg, P, sd, td, None, B, T, torch.zeros(B * T, 88, device=dev))
    np.testing.assert_allclose(ws.flow.cpu().numpy(), flows, rtol=2e-2)
    assert _rel(ws.xS.view(B, T, -1), xS) <= 3e-2


@pytest.mark.parametrize("strategy", ["batch_mode", "group"])
def test_encfm_engine_step_matches_oracle(strategy):
    """The whole training step of the asr_train.py family on the engine (PARITY config: f32 kernels,
    deterministic; the FM chain itself is bf16) vs oracle/ver5.py's ver5_step(kd_model="encfm") in
    float64 with the same router noise: losses rtol 2e-2 (the bf16 chain), the sampled steps exactly, and
    every trainable gradient relative Frobenius <= 5e-2 (the student encoder's gradients carry the bf16
    FM chain's data gradient)."""
    import test_step_parity_gpu as SP
    from oracle import ver5 as O
    from kdfm.config import sub_dims
    n_layers, B, N = 2, 2, 19200
    cfg, eng, wav, wl, tg, tgl, g = SP._build(n_layers, B, N, [19200, 16123], 12, [12, 7],
                                              sub=dict(kd_model="encfm", encfm_strategy=strategy))
    T = sub_dims(cfg, N // cfg.hop + 1)[-1][0]
    gum = -torch.empty(n_layers * B, cfg.router_max_steps).exponential_(generator=g).log()
    eng.encfm_gumbel = gum.cuda()
    ctx = eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True)
    losses = eng.losses.detach().cpu().clone()
    ews = ctx["ews"]
    steps = ews.steps.detach().cpu().clone()
    eng.backward(ctx)
    torch.cuda.synchronize()
    grads = eng.student.grads()
    ocfg, p32 = SP._oracle_params(cfg, eng)
    ocfg.kd_model, ocfg.encfm_strategy = "encfm", strategy
    p = {k: (v.double() if v.is_floating_point() else v) for k, v in p32.items()}
    names = O.trainable_names(p, cfg.version, cfg.use_diffkd)
    names = [k for k in names if not k.startswith(("tae.", "sproj.", "adapter.", "denoiser.", "fm_latent"))]
    for k in names:
        p[k] = p[k].clone().requires_grad_(True)
    out = O.ver5_step(p, wav.double(), wl, tg, tgl, ocfg, None, gumbel=list(gum.double().view(n_layers, B, -1)))
    assert torch.equal(steps.view(n_layers, B).long(), out["encfm"]["steps"])
    ref = torch.stack([out["loss"], out["ctc"], out["kl"], out["recon"], out["fm"]]).detach().float()
    torch.testing.assert_close(losses, ref, rtol=2e-2, atol=1e-3)
    og = torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
    bad = []
    for k, gr in zip(names, og):
        gr = torch.zeros_like(p[k]) if gr is None else gr
        if k.endswith(SP.ANALYTIC_ZERO) or gr.norm() == 0:
            continue
        r = _rel(grads[k], gr)
        if r > 5e-2:
            bad.append(f"{k}: {r:.3e}")
    assert not bad, bad
