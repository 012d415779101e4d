"""Where the one-kernel striding subsampling's bf16 y1 side output departs from the f32 conv1 (worst
elements with their (b, t1, f1, c) position, the f32 two-kernel conv1 value and the float64 reference)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kd-via-fm-in-asr_amd")]
from kdfm import kernels as K  # noqa: E402


def lens(n):
    return (n - 1) // 2 + 1


def main(C=88, Tm=57, ls=(57, 40, 23)):
    g = torch.Generator().manual_seed(C + Tm)
    B, Fq = 3, 80
    mel = torch.randn(B, Tm, Fq, generator=g)
    mel_len = torch.tensor(ls, dtype=torch.int64)
    len1 = lens(mel_len)
    len2 = lens(len1)
    w0 = torch.randn(C, 1, 3, 3, generator=g) * 0.3
    b0 = torch.randn(C, generator=g) * 0.1
    w2 = torch.randn(C, C, 3, 3, generator=g) * (1.0 / (3 * C ** 0.5))
    b2 = torch.randn(C, generator=g) * 0.1
    T1, F1 = lens(Tm), lens(Fq)
    T2, F2 = lens(T1), lens(F1)
    dev = "cuda"
    wp = torch.empty(K.subsample_fused_wprep_elems(C), device=dev, dtype=torch.bfloat16)
    K.subsample_fused_wprep(w0.cuda(), w2.cuda(), wp)
    y1 = torch.full((B * T1 * F1, C), float("nan"), device=dev).bfloat16()
    y2 = torch.full((B * T2 * F2, C), float("nan"), device=dev)
    K.subsample_fused(mel.cuda(), mel_len.cuda(), len1.cuda(), len2.cuda(), wp, b0.cuda(), b2.cuda(), y2, y1, B, Tm, Fq, C)
    y1b = torch.empty(B * T1 * F1, C, device=dev, dtype=torch.bfloat16)
    y1f = torch.empty(B * T1 * F1, C, device=dev)
    K.subsample_conv1(mel.cuda(), mel_len.cuda(), len1.cuda(), w0.cuda().view(C, 9), b0.cuda(), y1b, y1f, B, Tm, Fq, C)
    torch.cuda.synchronize()
    x = mel.clone()
    for b in range(B):
        x[b, mel_len[b]:] = 0
    r1 = F.relu(F.conv2d(x.double()[:, None], w0.double(), b0.double(), stride=2, padding=1))
    for b in range(B):
        r1[b, :, len1[b]:] = 0
    r1 = r1.permute(0, 2, 3, 1).reshape(B * T1 * F1, C)
    got = y1.float().cpu().double()
    d = (got - r1).abs()
    bad = d > 2.0 ** -7 * r1.abs() + 1e-6
    print(f"C={C} Tm={Tm}: {int(bad.sum())} of {bad.numel()} y1 elements off; max {d.max().item():.4e}; "
          f"two-kernel f32 conv1 vs ref max {(y1f.cpu().double() - r1).abs().max().item():.3e}")
    idx = torch.nonzero(bad)[:24]
    for r, c in idx.tolist():
        b, rem = divmod(r, T1 * F1)
        t1, f1 = divmod(rem, F1)
        print(f"  b={b} t1={t1} f1={f1} c={c}: fused {got[r, c].item():+.5f} ref {r1[r, c].item():+.5f} "
              f"f32 {y1f[r, c].item():+.5f}")
    rows_bad = torch.nonzero(bad.any(1)).flatten()
    t1s = sorted(set(((rows_bad % (T1 * F1)) // F1).tolist()))
    f1s = sorted(set((rows_bad % F1).tolist()))
    cs = sorted(set(torch.nonzero(bad.any(0)).flatten().tolist()))
    print("  t1 rows with errors:", t1s[:40], "f1:", f1s[:40], "channels:", cs[:40])


if __name__ == "__main__":
    main()
    main(176, 57, (57, 40, 23))
