"""Large-tile route vs the generic kdfm_gemm routes inside one bf16 XL step (same weights, inputs, deterministic):
relative Frobenius differences of every layer output and every gradient.  A correct route differs only by f32
accumulation order (~1e-6) plus the propagation of that through bf16 roundings downstream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import kdfm  # noqa: E402,F401
import torch  # noqa: E402


def run(big, sub, B, N):
    from test_step_parity_gpu import _build
    from kdfm import kernels as K
    K._BIG = big
    K._BIG_MIN_WORK = 0.0
    lens = [N] * B
    cfg, eng, wav, wl, tg, tgl, g = _build(2, B, N, lens, 12, [12] * B, sub=dict(sub, math="bf16"))
    from kdfm.config import sub_dims
    T = sub_dims(cfg, N // cfg.hop + 1)[-1][0]
    eps = torch.randn(2 * B * T, cfg.latent, generator=g)
    ctx = eng.forward(wav.cuda(), wl.cuda(), tg.cuda(), tgl.cuda(), train=True, eps=eps.cuda())
    losses = eng.losses.detach().cpu().clone()
    sf = ctx["sfeats"].detach().cpu().clone()
    eng.backward(ctx)
    torch.cuda.synchronize()
    return losses, sf, {k: v.detach().cpu().clone() for k, v in eng.student.grads().items()}


def main():
    from test_step_parity_gpu import XL, CL
    for name, sub in (("XL", XL), ("CL", CL)):
        a = run(True, sub, 8 if name == "XL" else 4, 96000)
        b = run(False, sub, 8 if name == "XL" else 4, 96000)
        fr = lambda x, y: ((x.double() - y.double()).norm() / y.double().norm().clamp_min(1e-30)).item()  # noqa: E731
        print(name, "losses", a[0].tolist(), b[0].tolist())
        for i in range(a[1].shape[0]):
            print(name, f"layer {i} output rel diff {fr(a[1][i], b[1][i]):.3e}")
        worst = sorted(((fr(a[2][k], b[2][k]), k) for k in a[2] if b[2][k].abs().max() > 0), reverse=True)[:12]
        for e, k in worst:
            print(name, f"grad {k}: {e:.3e}")


if __name__ == "__main__":
    main()
