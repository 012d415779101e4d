"""Locate wrong outputs of kdfm_subsample_conv2_dgrad against the float64 transposed conv: per parity
class, per channel block, fraction of matching entries.  usage: python tools/ss_dgrad_debug.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kdfm import kernels as K  # noqa: E402


def run(B, T1, F1, C):
    g = torch.Generator().manual_seed(5)
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    y1 = torch.rand(B, T1, F1, C, generator=g) + 0.1          # all positive: ReLU' = 1 everywhere
    dy2 = torch.randn(B, T2, F2, C, generator=g).bfloat16().float()
    w2 = (torch.randn(C, C, 3, 3, generator=g) * 0.1).bfloat16().float()
    x = torch.zeros(B, C, T1, F1, dtype=torch.float64, requires_grad=True)
    out = F.conv2d(x, w2.double(), stride=2, padding=1)
    (gx,) = torch.autograd.grad(out, x, dy2.double().permute(0, 3, 1, 2))
    ref = gx.permute(0, 2, 3, 1)
    wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
    K.subsample_dgrad_wprep(w2.cuda(), wt)
    dy1 = torch.full((B * T1 * F1, C), float("nan"), device="cuda")
    K.subsample_conv2_dgrad(dy2.cuda().reshape(-1, C), wt, y1.cuda().reshape(-1, C).bfloat16(), dy1, B, T1, F1, C)
    torch.cuda.synchronize()
    got = dy1.cpu().double().view(B, T1, F1, C)
    tol = 1e-3 * ref.abs().max().item()
    print(f"B={B} T1={T1} F1={F1} C={C}: rel {((got - ref).norm() / ref.norm()).item():.3e}", flush=True)
    for pt in (0, 1):
        for pf in (0, 1):
            gs, rs = got[:, pt::2, pf::2], ref[:, pt::2, pf::2]
            ok = ((gs - rs).abs() <= tol)
            line = f"  class pt={pt} pf={pf}: match {ok.double().mean().item():.3f}"
            for c0 in range(0, C, 32):
                line += f" | ch {c0}-{min(C, c0 + 32) - 1}: {ok[..., c0:c0 + 32].double().mean().item():.3f}"
            print(line, flush=True)
            if ok.double().mean().item() < 1:
                bad = (~ok).nonzero()[:4].tolist()
                for b_, t_, f_, c_ in bad:
                    print(f"    bad (b={b_}, t1={2 * t_ + pt}, f1={2 * f_ + pf}, c={c_}): got "
                          f"{gs[b_, t_, f_, c_].item():.4f} ref {rs[b_, t_, f_, c_].item():.4f}", flush=True)


run(1, 5, 4, 16)
run(2, 29, 11, 16)
run(2, 37, 13, 88)


def onehot(B, T1, F1, C):
    """dy2 nonzero at ONE source position (all channels 1): which dy1 positions does the kernel touch?"""
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    w2 = torch.ones(C, C, 3, 3)
    wt = torch.empty(K.subsample_dgrad_wprep_elems(C), device="cuda", dtype=torch.bfloat16)
    K.subsample_dgrad_wprep(w2.cuda(), wt)
    y1 = torch.ones(B, T1, F1, C)
    for t2 in range(T2):
        for f2 in range(F2):
            dy2 = torch.zeros(B, T2, F2, C)
            dy2[0, t2, f2, :] = 1.0
            x = torch.zeros(B, C, T1, F1, dtype=torch.float64, requires_grad=True)
            out = F.conv2d(x, w2.double(), stride=2, padding=1)
            (gx,) = torch.autograd.grad(out, x, dy2.double().permute(0, 3, 1, 2))
            ref = gx.permute(0, 2, 3, 1)[0, :, :, 0]
            dy1 = torch.full((B * T1 * F1, C), float("nan"), device="cuda")
            K.subsample_conv2_dgrad(dy2.cuda().reshape(-1, C), wt, y1.cuda().reshape(-1, C).bfloat16(), dy1, B, T1, F1,
                                    C)
            torch.cuda.synchronize()
            got = dy1.cpu().view(B, T1, F1, C)[0, :, :, 0]
            print(f"src (t2={t2}, f2={f2}):\n  ref {ref.tolist()}\n  got {got.tolist()}", flush=True)


onehot(1, 5, 4, 16)
