"""Precision diagnosis of the swin meta-encoder against tests/golden/kd_encfm_meta.npz: per-gradient
relative Frobenius errors with the GEMMs in bf16 and in exact f32 (the attention pair is bf16 either
way), and the fused attention pair alone against float64 at the fixture's shape (T=32, 2 heads of 60)."""
import os
import sys
from dataclasses import replace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kd-via-fm-in-asr_amd"), os.path.join(ROOT, "tests")]
import encfm_meta_fixture as FX  # noqa: E402
from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT, encfm_specs  # noqa: E402
from kdfm.encfm import encfm_backward, encfm_forward  # noqa: E402
from kdfm.fmmeta import MetaFMWorkspace  # noqa: E402


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def run(meta, math):
    z = FX.load()
    L, B, T = int(z["meta.L"]), int(z["meta.B"]), int(z["meta.T"])
    steps = tuple(int(x) for x in z["meta.steps"])
    cfg = replace(DEFAULT, n_layers=L, kd_model="encfm", encfm_meta=meta, encfm_dynamic=False,
                  encfm_steps_per_layer=steps, heads_student=2)
    dev = torch.device("cuda")
    P = {k: v.to(dev).contiguous() for k, v in FX.params(z, meta).items()}
    s, t, R = FX.inputs(z)
    sd = torch.stack([x.reshape(B * T, -1) for x in s]).to(dev).contiguous()
    td = torch.stack([x.reshape(B * T, -1) for x in t]).to(dev).contiguous()
    Rd = R.reshape(B * T, -1).to(dev).contiguous()
    G = {n: torch.zeros(shape, device=dev) for n, shape in encfm_specs(cfg)}
    ws = MetaFMWorkspace(cfg, B, T, dev)
    with K.mode(math, True):
        encfm_forward(cfg, P, sd, td, ws, train=True)
        dfeats = torch.empty(L * B * T, cfg.d_student, device=dev)
        encfm_backward(cfg, P, G, ws, dfeats, Rd, lambda fn, *keep: fn())
    torch.cuda.synchronize()
    pre = meta + "."
    print(f"== {meta} {math}: flow {ws.flow.cpu().tolist()} ref {z[pre + 'flow'].tolist()}  fm_out "
          f"{rel(ws.xS.view(B, T, -1), z[pre + 'fm_out']):.2e}")
    d = dfeats.view(L, B, T, -1)
    print("  d/ds:", [f"{rel(d[i], z[pre + f'grad.s{i}']):.2e}" for i in range(L)])
    for n, gr in G.items():
        print(f"  {n}: {rel(gr, z[pre + 'grad.' + n]):.2e}")


def attn_alone():
    B, H, T, dk = 2, 2, 32, 60
    d = H * dk
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = torch.randn(B * T, 3 * d, device="cuda", generator=g)
    q = qkv[:, :d].contiguous()
    do = torch.randn(B * T, d, device="cuda", generator=g)
    ppos = torch.zeros(2 * T - 1, d, device="cuda")
    lens = torch.full((B,), T, dtype=torch.int64, device="cuda")
    o = torch.empty(B * T, d, device="cuda")
    lse = torch.empty(B, H, T, device="cuda")
    sc = 1.0 / dk ** 0.5
    K.relpos_attn_fwd(q, q, qkv, ppos, lens, o, None, None, B, H, T, sc, 0.0, None, 0, lse=lse)
    ds, pd = K.attn_bwd2_saved(B, H, T, "cuda")
    rsum = torch.empty(B * H * T, device="cuda")
    dqu, dqv, dqkv = torch.empty_like(q), torch.empty_like(q), torch.zeros(B * T, 3 * d, device="cuda")
    K.relpos_attn_bwd2_dq(do, o, q, q, qkv, ppos, lse, lens, rsum, ds, pd, dqu, dqv, B, H, T, sc, 0.0, None, 0)
    K.relpos_attn_bwd2_dkv(do, q, ds, pd, lens, dqkv, B, H, T)
    torch.cuda.synchronize()
    x = qkv.double().cpu().requires_grad_(True)
    qq, kk, vv = (x[:, j * d:(j + 1) * d].reshape(B, T, H, dk).transpose(1, 2) for j in range(3))
    att = torch.softmax(qq @ kk.transpose(-1, -2) * sc, -1)
    oo = (att @ vv).transpose(1, 2).reshape(B * T, d)
    gx, = torch.autograd.grad(oo, x, do.double().cpu())
    print(f"== attention alone T={T} H={H} dk={dk}: o {rel(o, oo.detach()):.2e} dq {rel(dqu, gx[:, :d]):.2e} "
          f"dk {rel(dqkv[:, d:2 * d], gx[:, d:2 * d]):.2e} dv {rel(dqkv[:, 2 * d:], gx[:, 2 * d:]):.2e}")


if __name__ == "__main__":
    attn_alone()
    for meta in ("swin", "cnn"):
        for math in ("bf16", "f32"):
            run(meta, math)
