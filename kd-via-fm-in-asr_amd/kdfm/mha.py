"""Plain multi-head self-attention over the frames of each utterance (no positional terms, no masks):
the nn.MultiheadAttention core of the FM meta-encoders (asr_train.py SwinTransformerEncoder :844-866 and
ConformerBlock.mha :962-999), softmax(q k^T / sqrt(dk)) v with optional attention-weight dropout.

q | k | v come packed as the in-projection's (rows, 3d) output.  bf16 math: the fused attention pair
(attn_fused.hip forward with a zero positional table, attn_bwd.hip bwd2 backward: the forward keeps the
per-row log-sum-exp, the backward its bf16 dS / P-drop).  f32 math (parity): the unfused form of the
Conformer's f32 path -- scores and the P-weighted sum as batched kdfm_gemm products, the softmax (and
its dropout) in kdfm_relpos_softmax_fwd/bwd with a zero positional band -- exact f32 throughout.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from . import kernels as K


class MhaShape:
    """Shared (per B, T, d, H) buffers: the zero positional table / band, lengths, backward scratch."""

    def __init__(self, B, H, T, d, dev):
        self.B, self.H, self.T, self.d, self.dk = B, H, T, d, d // H
        if d % H or self.dk % 4 or self.dk > 64:
            raise ValueError(f"attention over {d} channels with {H} heads: the head dim must be a multiple of 4 "
                             "and <= 64")
        self.scale = 1.0 / math.sqrt(self.dk)
        self.fused = K.get_math() == "bf16"
        n = B * T
        f = lambda *s: torch.empty(*s, device=dev)  # noqa: E731
        self.lens = torch.full((B,), T, dtype=torch.int64, device=dev)
        self.dqu, self.dqv = f(n, d), f(n, d)
        if self.fused:
            self.ppos = torch.zeros(2 * T - 1, d, device=dev)
            self.ds, self.pd = K.attn_bwd2_saved(B, H, T, dev)
        else:
            self.bd = torch.zeros(B, H, T, 2 * T - 1, device=dev)
            self.ac, self.dpd, self.dac, self.dbd = f(B, H, T, T), f(B, H, T, T), f(B, H, T, T), f(B, H, T, 2 * T - 1)

    def saves(self, dev):
        """Per-evaluation saved state: lse (fused) or P and P-drop (unfused)."""
        B, H, T = self.B, self.H, self.T
        if self.fused:
            return {"lse": torch.empty(B, H, T, device=dev)}
        return {"P": torch.empty(B, H, T, T, device=dev), "Pd": torch.empty(B, H, T, T, device=dev)}


def mha_fwd(sh: MhaShape, sv, qkv, q, o, p, seed, rng_stream):
    """o (rows, d) = attention of qkv's q | k | v (q also as a contiguous copy in `q`)."""
    B, H, T, d, dk = sh.B, sh.H, sh.T, sh.d, sh.dk
    K.axpby(qkv[:, :d], None, q, 1.0, 0.0)
    if sh.fused:
        K.relpos_attn_fwd(q, q, qkv, sh.ppos, sh.lens, o, None, None, B, H, T, sh.scale, p, seed, rng_stream,
                          lse=sv["lse"])
        return
    K.gemm(q, qkv[:, d:], sh.ac, T, T, dk, d, 1, 1, 3 * d, T, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
           batch=(B, H), bA=(T * d, dk), bB=(T * 3 * d, dk), bC=(H * T * T, T * T))
    K.relpos_softmax_fwd(sh.ac, sh.bd, sh.lens, sv["P"], sv["Pd"] if p > 0 else None, B, H, T, sh.scale, p, seed,
                         rng_stream)
    Pd = sv["Pd"] if p > 0 else sv["P"]
    K.gemm(Pd, qkv[:, 2 * d:], o, T, dk, T, T, 1, 3 * d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * 3 * d, dk), bC=(T * d, dk))


def mha_bwd(sh: MhaShape, sv, qkv, q, o, do, dqkv, p, seed, rng_stream):
    """dqkv (rows, 3d) = d loss / d [q | k | v] given do = d loss / d o (overwritten)."""
    B, H, T, d, dk = sh.B, sh.H, sh.T, sh.d, sh.dk
    if sh.fused:
        K.relpos_attn_bwd2_dq(do, o, q, q, qkv, sh.ppos, sv["lse"], sh.lens, None, sh.ds, sh.pd, sh.dqu, sh.dqv,
                              B, H, T, sh.scale, p, seed, rng_stream)
        K.relpos_attn_bwd2_dkv(do, q, sh.ds, sh.pd, sh.lens, dqkv, B, H, T)
        K.axpby(sh.dqu, None, dqkv[:, :d], 1.0, 0.0)
        return
    Pm = sv["P"]
    Pd = sv["Pd"] if p > 0 else Pm
    # dPd = dO V^T
    K.gemm(do, qkv[:, 2 * d:], sh.dpd, T, T, dk, d, 1, 1, 3 * d, T, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
           batch=(B, H), bA=(T * d, dk), bB=(T * 3 * d, dk), bC=(H * T * T, T * T))
    K.relpos_softmax_bwd(Pm, sh.dpd, sh.dac, sh.dbd, B, H, T, sh.scale, p, seed, rng_stream)
    # dV = Pd^T dO, dQ = dAC K, dK = dAC^T Q (the softmax scale is inside dAC)
    K.gemm(Pd, do, dqkv[:, 2 * d:], T, dk, T, 1, T, d, 1, 3 * d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * d, dk), bC=(T * 3 * d, dk))
    K.gemm(sh.dac, qkv[:, d:], dqkv[:, :d], T, dk, T, T, 1, 3 * d, 1, 3 * d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * 3 * d, dk), bC=(T * 3 * d, dk))
    K.gemm(sh.dac, q, dqkv[:, d:], T, dk, T, 1, T, d, 1, 3 * d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * d, dk), bC=(T * 3 * d, dk))


__all__ = ["MhaShape", "mha_fwd", "mha_bwd"]
