"""Which kdfm_gemm route (and how fast) does a head-sized data-gradient product with a residual epilogue
take?  The NoiseAdapter backward's dx = dh W0 + dx_direct over the 16-layer stack (205,312 x 96 x 96,
heads.py _adapt_denoise_backward) showed up as a 327 us generic-tile launch in the step profile.
usage: python tools/route_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import _lib  # noqa: E402
from kdfm import kernels as K  # noqa: E402

dev = torch.device("cuda")
K.set_math("bf16")
n, L = 16 * 32 * 401, 96
flat = torch.randn(16384, device=dev)
W = flat[4:4 + L * L].view(L, L)
dh = torch.randn(n, L, device=dev)
R = torch.randn(n, L, device=dev)
dx = torch.empty(n, L, device=dev)
for label, kw in (("linear_dx + R", dict(R=R, rscale=1.0)), ("linear_dx", {})):
    K.linear_dx(dh, W, dx, **kw)
    torch.cuda.synchronize()
    route = K.ROUTES.get(int(_lib.lib().kdfm_gemm_last_route()), "?")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        K.linear_dx(dh, W, dx, **kw)
    e.record()
    torch.cuda.synchronize()
    print(f"{label:16s} route {route:12s} {1e3 * s.elapsed_time(e) / 20:8.1f} us", flush=True)
