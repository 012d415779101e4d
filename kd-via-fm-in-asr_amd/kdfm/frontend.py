"""Log-mel frontend: NeMo AudioToMelSpectrogramPreprocessor / FilterbankFeatures
(NeMo/nemo/collections/asr/modules/audio_preprocessing.py:61-304; leaf semantics SURVEY.md A.1).

Device pipeline (all libkdfm kernels):
  preemph_pad (dither, preemphasis, length mask, centre zero-pad 256)
  -> kdfm_logmel_fft: per frame (hop 160, Hann(400, periodic=False) centred in n_fft 512) a 512-point
     real FFT in f32 (one wave, LDS radix-2), |X|^2 of bins 0..256 and the Slaney mel filterbank
     (80 x 257, each filter over its nonzero bin range)
  -> log(x + 2^-24), per-feature normalisation over valid frames, zero beyond seq_len.
(KDFM_FRONTEND_FFT=0 selects the earlier DFT-as-GEMM chain: f32 MFMA GEMM against a (400 x 514)
[w cos | -w sin] basis, power, f32 filterbank GEMM.)
Output layout (B, T, 80) channels-last; the NeMo-facing module returns the (B, 80, T) view.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from . import kernels as K
from .config import Ver5Config


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, f / f_sp)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def slaney_filterbank(sr: int, n_fft: int, n_mels: int, fmin: float = 0.0, fmax: float | None = None) -> np.ndarray:
    """librosa.filters.mel(htk=False, norm='slaney') as NeMo builds it (audio_preprocessing.py:263-289)."""
    fmax = sr / 2 if fmax is None else fmax
    freqs = np.linspace(0, sr / 2, n_fft // 2 + 1)
    mel_pts = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_pts)
    ramps = mel_pts[:, None] - freqs[None, :]
    w = np.zeros((n_mels, n_fft // 2 + 1), dtype=np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_pts[2:n_mels + 2] - mel_pts[:n_mels]))[:, None]
    return w


def hann_symmetric(n: int) -> np.ndarray:
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / (n - 1))


def dft_basis(n_fft: int, win: int) -> np.ndarray:
    """(win, 2*(n_fft//2+1)) real basis: [w[k] cos(2pi f (k+off)/n) | -w[k] sin(...)], off = (n_fft-win)//2."""
    off = (n_fft - win) // 2
    F = n_fft // 2 + 1
    k = np.arange(win, dtype=np.float64)[:, None] + off
    f = np.arange(F, dtype=np.float64)[None, :]
    ang = 2.0 * np.pi * ((k * f) % n_fft) / n_fft
    w = hann_symmetric(win)[:, None]
    return np.concatenate([w * np.cos(ang), -w * np.sin(ang)], axis=1).astype(np.float32)


class FrontendConsts:
    """Device-resident constants (the preprocessor's `featurizer.fb` / `featurizer.window` buffers)."""

    def __init__(self, cfg: Ver5Config, device):
        self.cfg = cfg
        self.window = torch.tensor(hann_symmetric(cfg.win).astype(np.float32), device=device)
        self.fb = torch.tensor(slaney_filterbank(cfg.sample_rate, cfg.n_fft, cfg.nfilt), device=device)
        self.basis = torch.tensor(dft_basis(cfg.n_fft, cfg.win), device=device)
        j = np.arange(cfg.n_fft, dtype=np.float64)
        tw = np.stack([np.cos(2 * np.pi * j / cfg.n_fft), -np.sin(2 * np.pi * j / cfg.n_fft)], axis=1)
        self.twiddle = torch.tensor(tw.astype(np.float32), device=device)
        fbn = slaney_filterbank(cfg.sample_rate, cfg.n_fft, cfg.nfilt)
        lo = np.array([np.flatnonzero(r)[0] if r.any() else 0 for r in fbn], dtype=np.int32)
        hi = np.array([np.flatnonzero(r)[-1] + 1 if r.any() else 0 for r in fbn], dtype=np.int32)
        self.fb_lo = torch.tensor(lo, device=device)
        self.fb_hi = torch.tensor(hi, device=device)


def mel_frames(cfg: Ver5Config, n_samples: int) -> int:
    return n_samples // cfg.hop + 1


_FFT = __import__("os").environ.get("KDFM_FRONTEND_FFT", "1") == "1"


def frontend_forward(cfg: Ver5Config, consts: FrontendConsts, wav: torch.Tensor, wav_len: torch.Tensor,
                     mel_len: torch.Tensor, *, dither: float, seed=None, rng_stream: int = 0,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """wav (B, N) f32, wav_len (B,) i64 -> mel (B, T, nfilt) f32 (channels-last); mel_len must
    already hold wav_len // hop (kdfm_subsample_lengths)."""
    if not wav.is_cuda:
        raise _lib.KdfmError("frontend_forward needs a device tensor")
    B, N = wav.shape
    T = mel_frames(cfg, N)
    # algorithmic HBM bytes: read the f32 waveform, write the f32 log-mel
    with K.span("frontend", nbytes=4.0 * B * (N + T * cfg.nfilt)):
        return _frontend(cfg, consts, wav, wav_len, mel_len, dither, seed, rng_stream, out)


def _frontend(cfg, consts, wav, wav_len, mel_len, dither, seed, rng_stream, out):
    B, N = wav.shape
    pad = cfg.n_fft // 2
    T = mel_frames(cfg, N)
    F = cfg.n_fft // 2 + 1
    dev = wav.device
    xp = torch.empty(B, N + 2 * pad, device=dev)
    K.preemph_pad(wav.contiguous(), wav_len, xp, pad, cfg.preemph, dither, seed, rng_stream)
    mel = torch.empty(B * T, cfg.nfilt, device=dev)
    if _FFT and cfg.n_fft == 512:
        K.logmel_fft(xp, consts.window, consts.twiddle, consts.fb, consts.fb_lo, consts.fb_hi, mel, B, T, cfg.hop,
                     cfg.n_fft, cfg.win)
    else:
        spec = torch.empty(B * T, 2 * F, device=dev)
        off = (cfg.n_fft - cfg.win) // 2
        xv = xp[:, off:]
        K.gemm(xv, consts.basis, spec, T, 2 * F, cfg.win, cfg.hop, 1, 2 * F, 1, 2 * F, 1,
               amode=_lib.LD_KC, bmode=_lib.LD_XC, batch=(B, 1), bA=(N + 2 * pad, 0), bC=(T * 2 * F, 0), math="f32")
        power = torch.empty(B * T, F, device=dev)
        K.power_spectrum(spec, power)
        del spec
        K.linear(power, consts.fb, None, mel, math="f32")
    if out is None:
        out = torch.empty(B, T, cfg.nfilt, device=dev)
    K.logmel_normalize(mel, mel_len, out, B, T, cfg.nfilt, cfg.log_guard)
    return out


def specaugment_(cfg: Ver5Config, mel: torch.Tensor, mel_len: torch.Tensor, seed, rng_stream: int, mask_out=None,
                 uniforms=None):
    """NeMo's vectorized SpecAugment in place on mel (B, T, nfilt); uniforms: optional injected
    draws (parity mode, kernels.specaugment)."""
    B, T, nf = mel.shape
    K.specaugment(mel, mel_len, B, T, nf, cfg.freq_masks, cfg.freq_width, cfg.time_masks, cfg.time_width, seed,
                  rng_stream, mask_out, uniforms)
    return mel


__all__ = ["FrontendConsts", "frontend_forward", "specaugment_", "slaney_filterbank", "dft_basis", "mel_frames",
           "hann_symmetric", "math"]
