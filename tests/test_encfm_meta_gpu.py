"""The cnn / swin FM meta-encoders on the engine (kdfm/fmmeta.py) against (a) tests/golden/
kd_encfm_meta.npz, made from the reference's own FlowMatchingModule / SwinTransformerEncoder
(make_golden_encfm_meta.py; asr_train.py:844-1020, 1220-1377) -- in f32 math exactly, in bf16 math at the bf16 tolerances below --
and (b) the whole training step of the asr_train.py family with that meta-encoder (PARITY: f32 math,
deterministic, dropout off, fixed steps) vs oracle/ver5.py in float64: losses rtol 1e-4, every trainable
gradient relative Frobenius <= 1e-3."""
from dataclasses import replace

import numpy as np
import pytest
import torch

import encfm_meta_fixture as FX

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


# bf16-math tolerance on the parameter gradients (relative Frobenius).  cnn: the GEMMs' bf16 operands
# only (measured <= 1.6e-2).  swin: + the fused attention pair's bf16 P / dS, whose error the time
# embedding and the in / out projections collect through both chained steps (measured 3.0-5.8e-2 against
# the reference, 2-2.7e-2 with exact-f32 GEMMs around the same bf16 attention: profiles/r04/swin_diag.log).
BF16_GRAD_TOL = {"cnn": 3e-2, "swin": 8e-2, "conformer": 8e-2, "unet": 3e-2}


@pytest.mark.parametrize("math", ["f32", "bf16"])
@pytest.mark.parametrize("meta", ["cnn", "swin", "conformer", "unet"])
def test_meta_matches_reference(meta, math):
    """f32 math: every kernel on the path exact f32 (the attention in its unfused f32 form) -- losses rtol
    1e-5, FM output / feature gradients / parameter gradients relative Frobenius <= 1e-4 (BatchNorm's
    analytically-zero depthwise bias gradient: |g| < 1e-4, as the reference's own f32 residue), BatchNorm
    running statistics rtol 1e-4.  bf16 math: flow losses rtol 2e-2, FM output and feature gradients
    <= 3e-2, parameter gradients <= BF16_GRAD_TOL[meta]."""
    from kdfm import kernels as K
    from kdfm.config import DEFAULT, encfm_specs, meta_bn_specs
    from kdfm.encfm import encfm_backward, encfm_forward
    from kdfm.fmmeta import MetaFMWorkspace
    z = FX.load()
    L, B = int(z["meta.L"]), int(z["meta.B"])
    T = int(z.get(meta + ".meta.T", z["meta.T"]))   # (the unet fixture: its own even frame count)
    steps = tuple(int(x) for x in z["meta.steps"])
    cfg = replace(DEFAULT, n_layers=L, kd_model="encfm", encfm_meta=meta, encfm_dynamic=False,
                  encfm_steps_per_layer=steps, heads_student=2, dropout=0.0,
                  encfm_hidden=int(z.get(meta + ".meta.hidden", 128)))
    dev = torch.device("cuda")
    P = {k: v.to(dev).contiguous() for k, v in FX.params(z, meta).items()}
    s, t, R = FX.inputs(z, T=T)
    sd = torch.stack([x.reshape(B * T, -1) for x in s]).to(dev).contiguous()
    td = torch.stack([x.reshape(B * T, -1) for x in t]).to(dev).contiguous()
    Rd = R.reshape(B * T, -1).to(dev).contiguous()
    G = {n: torch.zeros(shape, device=dev) for n, shape in encfm_specs(cfg)}
    bn = {n: (torch.ones if n.endswith("running_var") else torch.zeros)(shape, device=dev)
          for n, shape in meta_bn_specs(cfg)}
    ws = MetaFMWorkspace(cfg, B, T, dev)
    with K.mode(math, True):
        encfm_forward(cfg, P, sd, td, ws, train=True, bn_running=bn)
        dfeats = torch.empty(L * B * T, cfg.d_student, device=dev)
        encfm_backward(cfg, P, G, ws, dfeats, Rd, lambda fn, *keep: fn())
    torch.cuda.synchronize()
    pre = meta + "."
    exact = math == "f32"
    np.testing.assert_allclose(ws.flow.cpu().numpy(), z[pre + "flow"], rtol=1e-5 if exact else 2e-2)
    np.testing.assert_allclose(ws.stats[2].item(), float(z[pre + "total"]), rtol=1e-5 if exact else 2e-2)
    tol = 1e-4 if exact else 3e-2
    assert _rel(ws.xS.view(B, T, -1), z[pre + "fm_out"]) <= tol
    d = dfeats.view(L, B, T, -1)
    for i in range(L):
        r = _rel(d[i], z[pre + f"grad.s{i}"])
        assert r <= tol, f"d/ds layer {i}: {r:.3e}"
    gtol = 1e-4 if exact else BF16_GRAD_TOL[meta]
    bad, worst = [], 0.0
    for n, gr in G.items():
        ref = z[pre + "grad." + n]
        if n.endswith("depthwise_conv.bias"):   # analytically zero (batch-statistics BatchNorm)
            assert gr.abs().max().item() < 1e-4 and np.abs(ref).max() < 1e-4, n
            continue
        r = _rel(gr, ref)
        worst = max(worst, r)
        if r > gtol:
            bad.append(f"{n}: {r:.3e}")
    print(f"{meta} {math}: worst parameter-gradient error {worst:.3e}")
    assert not bad, bad
    for n, v in bn.items():   # running statistics after sum(steps) module calls
        if exact:
            np.testing.assert_allclose(v.cpu().numpy(), z[pre + "buffer." + n], rtol=1e-4, atol=1e-6)
        else:
            assert _rel(v, z[pre + "buffer." + n]) <= 3e-2, n


@pytest.mark.parametrize("meta", ["cnn", "swin", "conformer", "unet"])
def test_meta_engine_step_matches_oracle(meta):
    import test_step_parity_gpu as SP
    from oracle import ver5 as O
    # (unet: 18 560 samples -> an even 30 subsampled frames, the only shapes UNet1D runs; base width 16)
    n_layers, B, N = 2, 2, (18560 if meta == "unet" else 19200)
    steps = (2, 3)
    extra = dict(encfm_hidden=16) if meta == "unet" else {}
    cfg, eng, wav, wl, tg, tgl, g = SP._build(n_layers, B, N, [N, 16123], 12, [12, 7],
                                              sub=dict(kd_model="encfm", encfm_dynamic=False, encfm_meta=meta,
                                                       encfm_steps_per_layer=steps, **extra))
    ctx = eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True)
    losses = eng.losses.detach().cpu().clone()
    eng.backward(ctx)
    torch.cuda.synchronize()
    grads = eng.student.grads()
    ocfg, p32 = SP._oracle_params(cfg, eng)
    ocfg.kd_model, ocfg.encfm_fixed, ocfg.encfm_meta = "encfm", steps, meta
    p = {k: (v.double() if v.is_floating_point() else v) for k, v in p32.items()}
    names = O.trainable_names(p, cfg.version, cfg.use_diffkd)
    names = [k for k in names if not k.startswith(("tae.", "sproj.", "adapter.", "denoiser.", "fm_latent", "router."))]
    for k in names:
        p[k] = p[k].clone().requires_grad_(True)
    out = O.ver5_step(p, wav.double(), wl, tg, tgl, ocfg, None)
    ref = torch.stack([out["loss"], out["ctc"], out["kl"], out["recon"], out["fm"]]).detach().float()
    torch.testing.assert_close(losses, ref, rtol=1e-4, atol=1e-5)
    og = torch.autograd.grad(out["loss"], [p[k] for k in names], allow_unused=True)
    bad = []
    for k, gr in zip(names, og):
        gr = torch.zeros_like(p[k]) if gr is None else gr
        if k.endswith(SP.ANALYTIC_ZERO) or gr.norm() == 0:
            continue
        if k.endswith("depthwise_conv.bias"):
            continue
        r = _rel(grads[k], gr)
        if r > 1e-3:
            bad.append(f"{k}: {r:.3e}")
    assert not bad, bad


@pytest.mark.parametrize("meta", ["swin", "conformer"])
def test_meta_workspace_follows_batch_shape(meta):
    """the engine keeps ONE meta-encoder workspace, the current batch shape's -- a new padded length
    replaces the previous one instead of stacking another full set of saved activations (allocated memory
    after steps at T1, T2, T1 stays within one workspace of the first step's peak) -- and an eval forward
    reports zero flow losses (asr_train.py:1363-1364: loss 0.0 outside training)."""
    import gc
    import weakref

    import test_step_parity_gpu as SP
    cfg, eng, wav, wl, tg, tgl, g = SP._build(2, 2, 19200, [19200, 16123], 12, [12, 7],
                                              sub=dict(kd_model="encfm", encfm_dynamic=False, encfm_meta=meta,
                                                       encfm_steps_per_layer=(2, 3)))
    wav2 = torch.cat([wav, wav[:, :6400]], 1)   # a longer padded batch: another T

    def step(w):
        ctx = eng.forward(w.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True)
        eng.backward(ctx)
        del ctx
        torch.cuda.synchronize()
        gc.collect()

    step(wav)
    first = next(iter(eng._encfm.values()))
    ref = weakref.ref(first)
    del first
    base = torch.cuda.memory_allocated()
    step(wav2)
    assert len(eng._encfm) == 1
    gc.collect()
    assert ref() is None, "the previous shape's workspace is still referenced"
    step(wav)
    assert len(eng._encfm) == 1
    grown = torch.cuda.memory_allocated() - base
    assert grown <= 0.05 * base + (1 << 20), (base, grown)
    eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=False)
    torch.cuda.synchronize()
    ws = next(iter(eng._encfm.values()))
    assert ws.flow.abs().max().item() == 0.0 and ws.stats[0].item() == 0.0
    assert torch.isfinite(ws.xS).all()


def test_conformer_meta_dropout_gradient_matches_finite_differences():
    """the conformer meta-encoder's dropout paths (FF activation / output masks with the 0.5 residual
    scale, the conv-output mask, the attention-weight dropout) had no test.  With dropout 0.1 and a fixed seed
    the engine's forward is a smooth deterministic function of the parameters (the masks come from the counter
    RNG), so its backward must equal central finite differences of its own forward: the directional derivative
    along a random direction over every flow_matching.* parameter, and along the meta-encoder's parameters only,
    within 2e-2 relative (f32 math, exact-f32 kernels).  A forward / backward mask or stream-index mismatch moves
    the gradient by O(p)."""
    from kdfm import kernels as K
    from kdfm.config import DEFAULT, encfm_specs, meta_bn_specs
    from kdfm.encfm import encfm_backward, encfm_forward
    from kdfm.fmmeta import MetaFMWorkspace
    z = FX.load()
    L, B, T = int(z["meta.L"]), int(z["meta.B"]), int(z["meta.T"])
    steps = tuple(int(x) for x in z["meta.steps"])
    cfg = replace(DEFAULT, n_layers=L, kd_model="encfm", encfm_meta="conformer", encfm_dynamic=False,
                  encfm_steps_per_layer=steps, heads_student=2, dropout=0.1)
    dev = torch.device("cuda")
    P = {k: v.to(dev).contiguous() for k, v in FX.params(z, "conformer").items()}
    s, t, R = FX.inputs(z)
    sd = torch.stack([x.reshape(B * T, -1) for x in s]).to(dev).contiguous()
    td = torch.stack([x.reshape(B * T, -1) for x in t]).to(dev).contiguous()
    Rd = R.reshape(B * T, -1).to(dev).contiguous()
    seed = torch.tensor([2024], dtype=torch.int64, device=dev)
    ws = MetaFMWorkspace(cfg, B, T, dev)

    def bn():
        return {n: (torch.ones if n.endswith("running_var") else torch.zeros)(shape, device=dev)
                for n, shape in meta_bn_specs(cfg)}

    def loss(Pm):
        encfm_forward(cfg, Pm, sd, td, ws, train=True, bn_running=bn(), seed=seed)
        torch.cuda.synchronize()
        return ws.stats[2].double().item() + (Rd.double() * ws.xS.double()).sum().item()

    with K.mode("f32", True):
        G = {n: torch.zeros(shape, device=dev) for n, shape in encfm_specs(cfg)}
        loss(P)
        dfeats = torch.empty(L * B * T, cfg.d_student, device=dev)
        encfm_backward(cfg, P, G, ws, dfeats, Rd, lambda fn, *keep: fn(), seed=seed)
        torch.cuda.synchronize()
        g = torch.Generator(device=dev).manual_seed(11)
        for subset in (lambda n: True, lambda n: n.startswith("flow_matching.meta_encoder.")):
            names = [n for n in G if subset(n)]
            v = {n: torch.randn(G[n].shape, device=dev, generator=g) * P[n].abs().mean().clamp_min(1e-3) for n in names}
            analytic = sum((G[n].double() * v[n].double()).sum().item() for n in names)
            eps = 1e-3
            plus = {n: (P[n] + eps * v[n]) if n in v else P[n] for n in P}
            minus = {n: (P[n] - eps * v[n]) if n in v else P[n] for n in P}
            fd = (loss(plus) - loss(minus)) / (2 * eps)
            assert abs(fd - analytic) <= 2e-2 * max(abs(analytic), abs(fd)), (len(names), fd, analytic)


def test_unet_refuses_odd_frame_counts():
    """UNet1D returns 2 floor(T / 2) frames, so at an odd T the reference's update x - v / S fails to broadcast
    (asr_train.py:1358); the engine refuses that shape with the reference's error text instead of training a
    different model."""
    from kdfm.config import DEFAULT
    from kdfm.fmmeta import MetaFMWorkspace
    cfg = replace(DEFAULT, n_layers=2, kd_model="encfm", encfm_meta="unet", encfm_dynamic=False,
                  encfm_steps_per_layer=(2, 3), encfm_hidden=16)
    with pytest.raises(ValueError, match="even frame count"):
        MetaFMWorkspace(cfg, 2, 31, torch.device("cuda"))
    MetaFMWorkspace(cfg, 2, 30, torch.device("cuda"))
