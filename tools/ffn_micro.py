"""Isolated timing of the fused LN-block kernels at the bench shape (12 832 rows): macaron FFN
forward / backward (student d=88 with dropout, teacher d=176 without), LN-fused projections and the
row-streaming products, against the unfused kdfm_gemm path they replace.  HIP events around N
back-to-back launches on one stream; prints one line per case (us per launch).
usage: python tools/ffn_micro.py [iters] [rows]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kd-via-fm-in-asr_amd")]

import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 12832
    dev = "cuda"
    seed = torch.tensor([12345], dtype=torch.int64, device=dev)
    K.set_math("bf16")
    for d, p in ((88, 0.1), (88, 0.0), (176, 0.0)):
        ff = 4 * d
        g = torch.Generator().manual_seed(d)
        W1 = (torch.randn(ff, d, generator=g) / d ** 0.5).to(dev)
        W2 = (torch.randn(d, ff, generator=g) / ff ** 0.5).to(dev)
        b1 = torch.zeros(ff, device=dev)
        b2 = torch.zeros(d, device=dev)
        lg, lb = torch.ones(d, device=dev), torch.zeros(d, device=dev)
        x = torch.randn(rows, d, device=dev)
        out = torch.empty_like(x)
        m, r = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
        img = K.ffn_img(W1, W2)
        fwd = lambda: K.ffn_fwd(x, lg, lb, 1e-5, img, b1, b2, out, m, r, ff, rscale=0.5, p_act=p, p_out=p,  # noqa
                                seed=seed, st_act=1, st_out=2)
        t_f = timeit(fwd, iters)
        bf = torch.bfloat16
        lnh, dl2h = torch.empty(rows, d, device=dev, dtype=bf), torch.empty(rows, d, device=dev, dtype=bf)
        ah, dhh = torch.empty(rows, ff, device=dev, dtype=bf), torch.empty(rows, ff, device=dev, dtype=bf)
        dx = torch.empty_like(x)
        part = torch.empty(K.layernorm_bwd_ws(rows, d), device=dev)
        bwd = lambda: K.ffn_bwd(x, x, m, r, lg, lb, img, b1, dx, lnh, ah, dl2h, dhh, part, ff, rscale=0.5,  # noqa
                                p_act=p, p_out=p, seed=seed, st_act=1, st_out=2)
        t_b = timeit(bwd, iters) if d <= 96 else float("nan")
        # unfused reference path (LN + up + down)
        ln = torch.empty_like(x)
        h = torch.empty(rows, ff, device=dev)
        a = torch.empty(rows, ff, device=dev)

        def unf():
            K.layernorm_fwd(x, lg, lb, ln, m, r, 1e-5)
            K.linear(ln, W1, b1, a, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE, Cpre=h, dropout_p=p, seed=seed,
                     rng_stream=1)
            K.linear(a, W2, b2, out, epi=_lib.EPI_RESID, R=x, rscale=0.5, dropout_p=p, seed=seed, rng_stream=2)
        t_u = timeit(unf, iters)
        flop = 4.0 * rows * d * ff
        print(f"ffn rows={rows} d={d} p={p}: fused fwd {t_f:7.1f} us ({flop / t_f / 1e6:6.1f} TFLOP/s)  bwd {t_b:7.1f} us  "
              f"| unfused fwd {t_u:7.1f} us", flush=True)
    # LN projections and row-streaming products at d=88
    d = 88
    x = torch.randn(rows, d, device=dev)
    lg, lb = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    Wq = (torch.randn(3 * d, d) / d ** 0.5).to(dev)
    bq = torch.zeros(3 * d, device=dev)
    u = torch.zeros(d, device=dev)
    qu, qv, qkv = torch.empty_like(x), torch.empty_like(x), torch.empty(rows, 3 * d, device=dev)
    m, r = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    iq = K.lnproj_img(0, Wq)
    print(f"ln_qkv_fwd d=88: {timeit(lambda: K.ln_qkv_fwd(x, lg, lb, 1e-5, iq, bq, u, u, qu, qv, qkv, m, r), iters):7.1f} us",
          flush=True)
    Wr = (torch.randn(d, d) / d ** 0.5).to(dev)
    ir = K.rowgemm_img(Wr)
    o = torch.empty_like(x)
    print(f"rowgemm resid d=88: {timeit(lambda: K.rowgemm(x, ir, o, epi=1, bias=u, R=x, p_out=0.1, st_out=3, seed=seed), iters):7.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
