"""Per-shape timing of the forward / data-gradient GEMMs of the ver5 step (bf16 math), to compare
kernel choices (run twice, e.g. with KDFM_SKINNY=0 and =1).  Each shape: 3 warm-ups, 20 timed
launches between HIP events; prints us/launch, TFLOP/s and unique-byte GB/s.
usage: python tools/shape_micro.py [filter]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402

flt = sys.argv[1] if len(sys.argv) > 1 else ""
dev = "cuda"
K.set_math("bf16")
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s):
    return torch.randn(*s, device=dev, generator=g)


def twin(W):
    """register a bf16 twin (+ transpose) for weight W, like FlatStore.enable_bf16_twins"""
    W = W.contiguous()
    r, c = W.shape
    flat = W.view(-1)
    _keep.append(flat)       # the registry holds a weak reference
    h = torch.empty(W.numel(), device=dev, dtype=torch.bfloat16)
    ht = torch.empty_like(h)
    K.register_bf16_twin(flat, h, ht, [(0, r, c)])
    K.cast_bf16(W.view(-1), h)
    K.cast_bf16_t(W.view(-1), ht, torch.tensor([[0, r, c, 0]], dtype=torch.int64, device=dev), 1, -(-(r * c) // 256))
    _keep.append((h, ht))
    return W


_keep = []


def bench(name, fn, flops, nbytes, reps=20):
    if flt and flt not in name:
        return
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    print(f"{name:44s} {us:8.1f} us {flops / us / 1e6:7.1f} TF/s {nbytes / us / 1e3:7.0f} GB/s", flush=True)


if os.environ.get("KDFM_DEBUG_TWIN"):
    Wdbg = twin(rnd(88, 88))
    print("twin lookup:", K.bf16_twin(Wdbg), K.bf16_twin(Wdbg, True), len(K._TWINS), flush=True)
M = 12832
for d in (88, 176):
    for (n_out, k_in, epi, tag) in [(4 * d, d, _lib.EPI_SILU, "ffn_up"), (d, 4 * d, _lib.EPI_RESID, "ffn_down"),
                                    (3 * d, d, 0, "qkv"), (d, d, _lib.EPI_RESID, "out/pw2"), (2 * d, d, 0, "pw1")]:
        x = rnd(M, k_in)
        W = twin(rnd(n_out, k_in) * 0.1)
        b = rnd(n_out)
        y = torch.empty(M, n_out, device=dev)
        R = rnd(M, n_out) if epi == _lib.EPI_RESID else None
        bench(f"fwd {tag} d{d} {M}x{n_out}x{k_in}",
              lambda: K.linear(x, W, b, y, epi=epi, R=R, rscale=0.5), 2 * M * n_out * k_in,
              4 * M * (n_out * (2 if R is not None else 1) + k_in))
        dy = rnd(M, n_out)
        dx = torch.empty(M, k_in, device=dev)
        bench(f"dx  {tag} d{d} {M}x{k_in}x{n_out}", lambda: K.linear_dx(dy, W, dx), 2 * M * n_out * k_in,
              4 * M * (n_out + k_in))
n, L, T = 205312, 96, 401
x = rnd(n, L)
y = torch.empty(n, L, device=dev)
R = rnd(n, L)
W = twin(rnd(L, L) * 0.1)
b = rnd(L)
Wf = twin(rnd(L, 3 * L) * 0.05)
bench("heads linear 205312x96x96 relu", lambda: K.linear(x, W, b, y, epi=_lib.EPI_RELU), 2 * n * L * L, 8 * n * L)
bench("heads linear 205312x96x96 resid", lambda: K.linear(x, W, b, y, epi=_lib.EPI_RESID, R=R, rscale=-0.125),
      2 * n * L * L, 12 * n * L)
bench("heads conv3 205312x96x288 relu", lambda: K.conv3(x, Wf, b, y, T, epi=_lib.EPI_RELU), 2 * n * L * 3 * L,
      8 * n * L)
bench("heads conv3 205312x96x288 resid", lambda: K.conv3(x, Wf, b, y, T, R=R, rscale=-1 / 9), 2 * n * L * 3 * L,
      12 * n * L)
xt = rnd(n, 176)
Wt = twin(rnd(96, 176) * 0.1)
bench("heads tae.enc 205312x96x176", lambda: K.linear(xt, Wt, b, y), 2 * n * 96 * 176, 4 * n * (96 + 176))
yt = torch.empty(n, 176, device=dev)
Wd = twin(rnd(176, 96) * 0.1)
bd = rnd(176)
bench("heads tae.dec 205312x176x96", lambda: K.linear(x, Wd, bd, yt), 2 * n * 96 * 176, 4 * n * (96 + 176))
