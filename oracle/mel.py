"""ORACLE (test infrastructure only — never imported by the product path).

numpy restatement of librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm='slaney')
as pinned by NeMo/requirements/requirements_asr.txt:9 (librosa>=0.10.1) and called from NeMo's
FilterbankFeatures (constructed at NeMo/nemo/collections/asr/modules/audio_preprocessing.py:263-289).
librosa is not installed here, so this follows its published algorithm (Slaney auditory toolbox
mel scale: linear below 1 kHz, log above).  Parity unpinned against librosa itself: no reference
fixture holds filterbank values.
"""
from __future__ import annotations

import numpy as np


def hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr=16000, n_fft=512, n_mels=80, fmin=0.0, fmax=8000.0) -> np.ndarray:
    """(n_mels, n_fft//2+1) float32 Slaney-normalised triangular filters."""
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    weights = np.zeros((n_mels, n_fft // 2 + 1), dtype=np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights
