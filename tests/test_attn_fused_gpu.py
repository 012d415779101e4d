"""Fused relative-position attention forward (kdfm_relpos_attn_fwd, bf16) against (a) the unfused
bf16 path the encoder uses in parity mode's structure (AC / BD GEMMs + relpos_softmax_fwd + PV GEMM)
and (b) torch fp32 on the same bf16-rounded operands.

The fused kernel rounds the CENTRED keys / values to bf16 (K_j - kc, V_j - vc; kc / vc = the mean of the
utterance's first min(length, 16) rows, csrc/attn_centre.h), so the P references are formed from the same
centred keys (softmax is invariant to the shift; the bf16 rounding is then the kernel's).

Tolerances: P within 2e-3 absolute of the fp32 reference (scores from identical bf16 operands,
different f32 accumulation order; P <= 1); the dropout mask identical to the unfused kernel's
(same counter-RNG index); O within 1e-2 of max |O| (both round P_drop to bf16 for the PV MFMA)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def kv_centred(qkv, lens, B, T, d):
    """qkv with each utterance's keys and values shifted by the fused attention's centre (attn_centre.h):
    the mean of its first n rows, n = min(length, 16) rounded down to a power of two."""
    out = qkv.clone().view(B, T, 3 * d)
    for bi in range(B):
        L = min(int(lens[bi]), T)
        n = 1 << (min(L, 16).bit_length() - 1) if L > 0 else 0
        if n:
            out[bi, :, d:] -= out[bi, :n, d:].sum(0) / n
    return out.view(B * T, 3 * d)


def _unfused(K, _lib, qu, qv, qkv, ppos, lens, B, H, T, d, p, seed):
    dk = d // H
    npos = 2 * T - 1
    ac = torch.empty(B, H, T, T, device="cuda")
    K.gemm(qu, qkv[:, d:], ac, T, T, dk, d, 1, 1, 3 * d, T, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
           batch=(B, H), bA=(T * d, dk), bB=(T * 3 * d, dk), bC=(H * T * T, T * T), math="bf16")
    bd = torch.empty(B, H, T, npos, device="cuda")
    K.gemm(qv, ppos, bd, T, npos, dk, d, 1, 1, d, npos, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
           batch=(B, H), bA=(T * d, dk), bB=(0, dk), bC=(H * T * npos, T * npos), math="bf16")
    P = torch.empty(B, H, T, T, device="cuda")
    Pd = torch.empty(B, H, T, T, device="cuda") if p > 0 else P
    K.relpos_softmax_fwd(ac, bd, lens, P, Pd if p > 0 else None, B, H, T, 1.0 / math.sqrt(dk), p, seed, 11)
    o = torch.empty(B * T, d, device="cuda")
    K.gemm(Pd, qkv[:, 2 * d:], o, T, dk, T, T, 1, 3 * d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * 3 * d, dk), bC=(T * d, dk), math="bf16")
    return P, Pd, o


def _torch_ref_P(qu, qv, qkv, ppos, lens, B, H, T, d):
    dk = d // H
    q_u = _bf(qu).view(B, T, H, dk).permute(0, 2, 1, 3)
    q_v = _bf(qv).view(B, T, H, dk).permute(0, 2, 1, 3)
    k = _bf(qkv[:, d:2 * d]).reshape(B, T, H, dk).permute(0, 2, 1, 3)
    pp = _bf(ppos).view(2 * T - 1, H, dk).permute(1, 0, 2)            # (H, 2T-1, dk)
    ac = q_u @ k.transpose(-1, -2)
    bdf = torch.einsum("bhic,hrc->bhir", q_v, pp)                     # (B,H,T,2T-1)
    idx = (T - 1 - torch.arange(T, device="cuda")[:, None] + torch.arange(T, device="cuda")[None, :])
    bd = torch.gather(bdf, 3, idx.expand(B, H, T, T))
    s = (ac + bd) / math.sqrt(dk)
    keym = torch.arange(T, device="cuda")[None, :] < lens[:, None]       # (B, T)
    s = s.masked_fill(~keym[:, None, None, :], float("-inf"))
    P = torch.softmax(s, -1)
    rowm = keym[:, None, :, None]
    return torch.where(rowm, P, torch.zeros_like(P))


@pytest.mark.parametrize("B,H,T,d,p", [(3, 2, 401, 88, 0.0), (2, 4, 401, 176, 0.1), (2, 2, 77, 88, 0.1),
                                       (2, 4, 130, 176, 0.0), (1, 2, 64, 88, 0.0),
                                       # head dim 64 (FastConformer d=512, 8 heads)
                                       (2, 8, 201, 512, 0.1), (2, 2, 77, 128, 0.0)])
def test_fused_attention_matches(B, H, T, d, p):
    from kdfm import _lib
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(T + d)
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device="cuda", generator=g)
    qu = torch.randn(rows, d, device="cuda", generator=g)
    qv = torch.randn(rows, d, device="cuda", generator=g)
    ppos = torch.randn(2 * T - 1, d, device="cuda", generator=g)
    lens = torch.tensor([T] + [max(1, T - 17 * (i + 1)) for i in range(B - 1)], dtype=torch.int64, device="cuda")
    seed = torch.tensor([1234567], dtype=torch.int64, device="cuda")
    qkv_c = kv_centred(qkv, lens, B, T, d)
    P_u, Pd_u, _ = _unfused(K, _lib, qu, qv, qkv_c, ppos, lens, B, H, T, d, p, seed)
    _, _, o_u = _unfused(K, _lib, qu, qv, qkv, ppos, lens, B, H, T, d, p, seed)
    P_f = torch.empty(B, H, T, T, device="cuda")
    Pd_f = torch.empty(B, H, T, T, device="cuda") if p > 0 else None
    o_f = torch.empty(rows, d, device="cuda")
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o_f, P_f, Pd_f, B, H, T, 1.0 / math.sqrt(d // H), p, seed, 11)
    torch.cuda.synchronize()
    P_ref = _torch_ref_P(qu, qv, qkv_c, ppos, lens, B, H, T, d)
    assert (P_f - P_ref).abs().max().item() < 2e-3
    assert (P_f - P_u).abs().max().item() < 2e-3
    if p > 0:
        live = P_u > 1e-6
        assert torch.equal((Pd_f[live] == 0), (Pd_u[live] == 0))
        assert (Pd_f - Pd_u).abs().max().item() < 2e-3 / (1 - p)
    err = (o_f - o_u).abs().max().item()
    assert err <= 1e-2 * o_u.abs().max().item(), err
    # padded query rows produce zero output
    for bi in range(B):
        assert o_f.view(B, T, d)[bi, int(lens[bi]):].abs().max().item() == 0 if int(lens[bi]) < T else True


def test_fused_attention_no_P(K=None):
    """teacher mode (no P / P_drop outputs): single-pass online softmax, same O as the two-pass
    mode up to bf16 rounding of the unnormalised probabilities (1e-2 of max |O|)"""
    from kdfm import kernels as K
    g = torch.Generator(device="cuda").manual_seed(3)
    B, H, T, d = 2, 4, 401, 176
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device="cuda", generator=g)
    qu = torch.randn(rows, d, device="cuda", generator=g)
    qv = torch.randn(rows, d, device="cuda", generator=g)
    ppos = torch.randn(2 * T - 1, d, device="cuda", generator=g)
    lens = torch.tensor([T, 300], dtype=torch.int64, device="cuda")
    o1 = torch.empty(rows, d, device="cuda")
    o2 = torch.empty(rows, d, device="cuda")
    P = torch.empty(B, H, T, T, device="cuda")
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o1, None, None, B, H, T, 0.15, 0.0, None, 0)
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o2, P, None, B, H, T, 0.15, 0.0, None, 0)
    torch.cuda.synchronize()
    assert (o1 - o2).abs().max().item() <= 1e-2 * o2.abs().max().item()
    assert o1.view(B, T, d)[1, 300:].abs().max().item() == 0
