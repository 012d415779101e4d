"""Per-kernel times of the log-mel frontend at the bench shape (B=32 x 16 s): pre-emphasis / pad, the
per-frame FFT + mel kernel, the log + normalisation.  usage: python tools/frontend_micro.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kd-via-fm-in-asr_amd"))
import torch  # noqa: E402

from kdfm import kernels as K  # noqa: E402
from kdfm.config import DEFAULT as cfg  # noqa: E402
from kdfm.frontend import FrontendConsts, mel_frames  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda")
B, N = 32, 256000
T = mel_frames(cfg, N)
pad = cfg.n_fft // 2
fe = FrontendConsts(cfg, dev)
wav = 0.1 * torch.randn(B, N, device=dev)
wl = torch.full((B,), N, dtype=torch.int64, device=dev)
ml = torch.empty(B, dtype=torch.int64, device=dev)
K.subsample_lengths(wl, ml, None, None, cfg.hop)
xp = torch.empty(B, N + 2 * pad, device=dev)
mel = torch.empty(B * T, cfg.nfilt, device=dev)
out = torch.empty(B, T, cfg.nfilt, device=dev)
steps = {
    "preemph_pad": lambda: K.preemph_pad(wav, wl, xp, pad, cfg.preemph, 0.0, None, 0),
    "logmel_fft": lambda: K.logmel_fft(xp, fe.window, fe.twiddle, fe.fb, fe.fb_lo, fe.fb_hi, mel, B, T, cfg.hop,
                                       cfg.n_fft, cfg.win),
    "logmel_normalize": lambda: K.logmel_normalize(mel, ml, out, B, T, cfg.nfilt, cfg.log_guard),
}
for name, fn in steps.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{name:18s} {1e3 * s.elapsed_time(e) / reps:8.1f} us", flush=True)
