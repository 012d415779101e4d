"""Fused attention backward (v1 and bwd2) against float64 at short utterances (T < 64: one key block) and
scaled inputs (large logits): rel. Frobenius per gradient."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kd-via-fm-in-asr_amd"), os.path.join(ROOT, "tests")]
import test_attn_bwd_gpu as A  # noqa: E402
from kdfm import kernels as K  # noqa: E402

CM = float(os.environ.get("KCM", "0"))   # common-mode offset added to every key / value (per channel)
for (B, H, T, d) in [(2, 8, 26, 512), (2, 2, 26, 88), (2, 8, 201, 512)]:
    for scale in (1.0, 3.0):
        qkv, qu, qv, ppos, do, lens = A._inputs(B, H, T, d, T + d)
        lens = torch.tensor([T, max(1, T - 6)], dtype=torch.int64, device="cuda")
        qkv, qu, qv, ppos = qkv * scale, qu * scale, qv * scale, ppos * scale
        if CM:
            g = torch.Generator(device="cuda").manual_seed(1)
            qkv[:, d:] += CM * torch.randn(1, 2 * d, device="cuda", generator=g)
        seed = torch.tensor([99], dtype=torch.int64, device="cuda")
        _, _, dqu, dqv, dk_, dv_, dpos = A._fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, 0.0, seed)
        ref = A._torch_grads(qkv, qu, qv, ppos, do, lens, B, H, T, d)
        r1 = [A._rel(g, w) for g, w in zip((dqu, dqv, dk_, dv_, dpos), ref)]
        _, _, dS, Pd, dqu, dqv, dk_, dv_, dpos = A._bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, 0.0, seed)
        r2 = [A._rel(g, w) for g, w in zip((dqu, dqv, dk_, dv_, dpos), ref)]
        print(f"B={B} H={H} T={T} d={d} x{scale} cm={CM}: bwd1 " + " ".join(f"{v:.1e}" for v in r1) + " | bwd2 " +
              " ".join(f"{v:.1e}" for v in r2))
