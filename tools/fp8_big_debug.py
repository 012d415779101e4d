"""Localise an MX fp8 large-tile GEMM error: kernels.linear on the fp8 route against float64 of the dequantised
operands, with block exponents (a) uniform, (b) varying by row only, (c) varying by 32-k block only, (d) random."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
sys.path.insert(0, ROOT)
import kdfm  # noqa: E402,F401
import torch  # noqa: E402
from kdfm import kernels as K  # noqa: E402


def mx(t):
    x = t.double().reshape(t.shape[0], -1, 32)
    amax = x.abs().max(2, keepdim=True).values
    e = torch.ceil(torch.log2(amax.clamp_min(1e-300) / 448.0))
    e = torch.where(amax > 0, e, torch.full_like(e, -127.0)).clamp(-127, 127)
    q = (x / torch.pow(2.0, e)).float().to(torch.float8_e4m3fn).reshape(t.shape)
    return (q.double().reshape(t.shape[0], -1, 32) * torch.pow(2.0, e)).reshape(t.shape)


def case(name, x, W):
    M, Kd = x.shape
    N = W.shape[0]
    y = torch.empty(M, N, device="cuda")
    K._State.fp8 = True
    n = [0]
    orig = K.call

    def call(name, *a):
        n[0] += name == "kdfm_gemm_big_fp8"
        return orig(name, *a)
    K.call = call
    try:
        K.linear(x, W, None, y)
    finally:
        K._State.fp8 = False
        K.call = orig
    assert n[0] == 1, "the fp8 route was not taken"
    torch.cuda.synchronize()
    ref = mx(x) @ mx(W).t()
    # the kernel's own MX copies (scratch slot 0: x bytes, x scales, W bytes, W scales) against the torch restatement
    buf = max(K._SCRATCH.values(), key=lambda t: t.numel()).view(torch.uint8)
    off = 0
    deq = []
    for t in (x, W):
        r, kc = t.shape
        q = buf[off: off + r * kc].view(r, kc).clone()
        off += r * kc
        nsc = r * kc // 32
        sc = buf[off: off + nsc].clone()
        off += -(-nsc // 16) * 16
        e = sc.view(kc // 128, r, 4).permute(1, 0, 2).reshape(r, kc // 32).long() - 127
        dq = (q.view(torch.float8_e4m3fn).double().view(r, -1, 32) * torch.pow(2.0, e.double()).unsqueeze(2)).view(r, kc)
        dmax = (dq - mx(t)).abs().max().item()
        print(f"   kernel MX copy vs torch restatement: max |diff| {dmax:.3g}", flush=True)
        deq.append(dq)
    kref = deq[0] @ deq[1].t()
    print(f"   kernel vs its own MX copies: max rel {((y.double() - kref).abs() / (deq[0].abs() @ deq[1].abs().t() + 1e-30)).max().item():.3g}", flush=True)
    err = (y.double() - ref).abs()
    rel = err / (mx(x).abs() @ mx(W).abs().t() + 1e-30)
    bad = rel > 1e-4
    rows = bad.any(1).nonzero().flatten().tolist()
    cols = bad.any(0).nonzero().flatten().tolist()
    print(f"{name}: max rel {rel.max().item():.3g}; bad rows {len(rows)} (first {rows[:8]}), bad cols {len(cols)} "
          f"(first {cols[:8]})", flush=True)
    if rows:
        r, c = rows[0], cols[0]
        # which 32-k blocks would fix it: solve per-block factor guess by comparing partial sums
        xb, wb = mx(x)[r].reshape(-1, 32), mx(W)[c].reshape(-1, 32)
        parts = (xb * wb).sum(1)
        print(f"   C[{r},{c}] got {y[r, c].item():.6g} ref {ref[r, c].item():.6g}; per-block partials "
              f"{[round(p, 4) for p in parts.tolist()]}", flush=True)


def main():
    K.set_math("bf16")
    K._BIG_MIN_WORK = 0.0
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, Kd = 512, 512, 512

    def ints(r, c):
        t = torch.randint(-3, 4, (r, c), device=dev, generator=g).float()
        t.view(r, -1, 32)[:, :, 0] = 4.0
        return t
    x, W = ints(M, Kd), ints(N, Kd)
    case("uniform exponents", x, W)
    rs = torch.pow(2.0, torch.randint(-3, 4, (M, 1), device=dev, generator=g).float())
    ws = torch.pow(2.0, torch.randint(-3, 4, (N, 1), device=dev, generator=g).float())
    case("row-varying exponents", x * rs, W * ws)
    kb = torch.pow(2.0, torch.randint(-3, 4, (1, Kd // 32, 1), device=dev, generator=g).float())
    case("k-block-varying exponents (A only)", (x.view(M, -1, 32) * kb).view(M, Kd), W)
    case("k-block-varying exponents (B only)", x, (W.view(N, -1, 32) * kb).view(N, Kd))
    kb2 = torch.pow(2.0, torch.randint(-3, 4, (1, Kd // 32, 1), device=dev, generator=g).float())
    case("k-block-varying exponents (A and B, independent)", (x.view(M, -1, 32) * kb).view(M, Kd),
         (W.view(N, -1, 32) * kb2).view(N, Kd))
    ea = torch.pow(2.0, torch.randint(-3, 4, (M, Kd // 32, 1), device=dev, generator=g).float())
    eb = torch.pow(2.0, torch.randint(-3, 4, (N, Kd // 32, 1), device=dev, generator=g).float())
    case("per-(row, block) exponents, integer data", (x.view(M, -1, 32) * ea).view(M, Kd),
         (W.view(N, -1, 32) * eb).view(N, Kd))

    def e4(r, c):   # random e4m3 values with the block max pinned at 448 (so the block exponent is 0)
        t = (torch.randn(r, c, device=dev, generator=g) * 100).clamp(-440, 440).to(torch.float8_e4m3fn).float()
        t.view(r, -1, 32)[:, :, 5] = 448.0
        return t
    case("random e4m3 values, exponent 0", e4(M, Kd), e4(N, Kd))
    xa, wa = e4(M, Kd), e4(N, Kd)
    case("random e4m3 values, per-(row, block) exponents", (xa.view(M, -1, 32) * ea).view(M, Kd),
         (wa.view(N, -1, 32) * eb).view(N, Kd))
    case("random", torch.randn(M, Kd, device=dev, generator=g), torch.randn(N, Kd, device=dev, generator=g))


if __name__ == "__main__":
    main()
