"""Fused relative-position attention backward (kdfm_relpos_attn_bwd, csrc/attn_bwd.hip, bf16 MFMA)
against (a) float64 torch autograd of NeMo's rel-pos attention (Appendix A.7: scores = ((q+u)K^T +
rel_shift((q+v)Ppos^T)) / sqrt(dk), key mask, softmax, rows of padded queries zeroed, O = P V) with
no dropout, and (b) the unfused f32 path (dPd GEMM + relpos_softmax_bwd + five batched GEMMs) on
the saved P of the two-pass forward with attention dropout 0.1 (same counter-RNG mask).  The fused
backward reads no f32 probabilities: its dQ kernel recomputes them from the single-pass forward's
per-row log-sum-exp, its dK/dV and dPpos kernels form P = p~ exp(m_blk - lse) from the forward's bf16
unnormalised p~ and per-64-key-block running maxima; lse and that reconstruction are checked against
float64 too (P: max |diff| <= 1e-2 * max P + 1e-3, bf16 p~).

Tolerances: relative Frobenius error per gradient (dQu, dQv, dK, dV, dPpos) <= 2e-2 against float64
(bf16 operands, f32 accumulation) and <= 2e-2 against the unfused f32 kernels; padded keys get
exactly zero dK / dV; two runs are bitwise identical (no atomics).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _inputs(B, H, T, d, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device="cuda", generator=g)
    qu = torch.randn(rows, d, device="cuda", generator=g)
    qv = torch.randn(rows, d, device="cuda", generator=g)
    ppos = torch.randn(2 * T - 1, d, device="cuda", generator=g)
    do = torch.randn(rows, d, device="cuda", generator=g)
    lens = torch.tensor([T] + [max(1, T - 23 * (i + 1)) for i in range(B - 1)], dtype=torch.int64, device="cuda")
    return qkv, qu, qv, ppos, do, lens


def _fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed):
    """single-pass forward (O + lse, p~, m_blk), then the fused backward; returns ((lse, p~, m_blk), O, grads...)"""
    dk = d // H
    lse, pt, mblk = K.attn_saved(B, H, T, "cuda")
    o = torch.empty(B * T, d, device="cuda")
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, None, None, B, H, T, 1.0 / math.sqrt(dk), p, seed, 11, lse=lse,
                      p_tilde=pt, m_blk=mblk)
    dqu = torch.empty(B * T, d, device="cuda")
    dqv = torch.empty_like(dqu)
    dqkv = torch.zeros(B * T, 3 * d, device="cuda")
    dpos = torch.empty(2 * T - 1, d, device="cuda")
    K.relpos_attn_bwd(do, o, qu, qv, qkv, ppos, lse, pt, mblk, lens, dqu, dqv, dqkv, dpos, B, H, T,
                      1.0 / math.sqrt(dk), p, seed, 11)
    torch.cuda.synchronize()
    return (lse, pt, mblk), o, dqu, dqv, dqkv[:, d:2 * d], dqkv[:, 2 * d:], dpos


def _torch_grads(qkv, qu, qv, ppos, do, lens, B, H, T, d):
    dk = d // H
    f = lambda t: t.double().detach().clone().requires_grad_(True)  # noqa: E731
    q_u, q_v, k, v, pp = f(qu), f(qv), f(qkv[:, d:2 * d]), f(qkv[:, 2 * d:]), f(ppos)
    sh = lambda t: t.view(B, T, H, dk).permute(0, 2, 1, 3)  # noqa: E731
    ac = sh(q_u) @ sh(k).transpose(-1, -2)
    bdf = torch.einsum("bhic,hrc->bhir", sh(q_v), pp.view(2 * T - 1, H, dk).permute(1, 0, 2))
    idx = (T - 1 - torch.arange(T, device="cuda")[:, None] + torch.arange(T, device="cuda")[None, :])
    bd = torch.gather(bdf, 3, idx.expand(B, H, T, T))
    s = (ac + bd) / math.sqrt(dk)
    keym = torch.arange(T, device="cuda")[None, :] < lens[:, None]
    s = s.masked_fill(~keym[:, None, None, :], float("-inf"))
    _torch_grads.lse = torch.logsumexp(s, -1).detach()
    P = torch.softmax(s, -1)
    P = torch.where(keym[:, None, :, None], P, torch.zeros_like(P))
    _torch_grads.P = P.detach()
    O = (P @ sh(v)).permute(0, 2, 1, 3).reshape(B * T, d)
    loss = (O * do.double()).sum()
    return torch.autograd.grad(loss, [q_u, q_v, k, v, pp])


@pytest.mark.parametrize("B,H,T,d", [(3, 2, 401, 88), (2, 4, 130, 176), (2, 2, 77, 88),
                                     # head dim 64 (FastConformer d=512, 8 heads; fast-conformer_ctc_bpe.yaml:94-143)
                                     (2, 8, 201, 512), (2, 2, 77, 128)])
def test_attn_bwd_matches_float64(B, H, T, d):
    from kdfm import kernels as K
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, T + d)
    seed = torch.tensor([99], dtype=torch.int64, device="cuda")
    (lse, pt, mblk), _, dqu, dqv, dk_, dv_, dpos = _fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, 0.0, seed)
    ref = _torch_grads(qkv, qu, qv, ppos, do, lens, B, H, T, d)
    for name, got, want in zip(("dQu", "dQv", "dK", "dV", "dPpos"), (dqu, dqv, dk_, dv_, dpos), ref):
        assert _rel(got, want) <= 2e-2, (name, _rel(got, want))
    # the forward's per-row log-sum-exp (valid rows) against float64 -- of the centred keys' scores
    # (csrc/attn_centre.h: lse - scale qu_i . kc); rows past the length are 3e38
    from test_attn_fused_gpu import kv_centred
    kc = (qkv - kv_centred(qkv, lens, B, T, d))[:, d:2 * d].double().view(B, T, H, d // H)
    shift = (qu.double().view(B, T, H, d // H) * kc).sum(-1).permute(0, 2, 1) / math.sqrt(d // H)
    want = _torch_grads.lse - shift
    for bi in range(B):
        L = int(lens[bi])
        err = (lse[bi, :, :L].double().cpu() - want[bi, :, :L].cpu()).abs().max().item()
        assert err <= 2e-2 * max(1.0, want[bi, :, :L].abs().max().item()), (bi, err)
        if L < T:
            assert (lse[bi, :, L:] == 3.0e38).all()
        # P = p~ exp(m_blk[key block] - lse) on the valid square
        kb = torch.arange(L, device="cuda") // 64
        prec = pt[bi, :, :L, :L].float() * torch.exp(mblk[bi, :, :L][:, :, kb] - lse[bi, :, :L, None])
        pw = _torch_grads.P[bi, :, :L, :L]
        perr = (prec.double() - pw).abs().max().item()
        assert perr <= 1e-2 * pw.abs().max().item() + 1e-3, (bi, perr)
    # keys past an utterance's length receive no gradient
    for bi in range(B):
        L = int(lens[bi])
        if L < T:
            assert dk_.view(B, T, d)[bi, L:].abs().max().item() == 0.0
            assert dv_.view(B, T, d)[bi, L:].abs().max().item() == 0.0


def _unfused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed):
    """The unfused f32 chain on the two-pass forward's saved P and P_drop (same counter-RNG dropout mask):
    returns (O, (dQu, dQv, dK, dV, dPpos))."""
    from kdfm import _lib
    dk = d // H
    npos = 2 * T - 1
    P = torch.empty(B, H, T, T, device="cuda")
    Pd = torch.empty_like(P)
    o = torch.empty(B * T, d, device="cuda")
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, P, Pd, B, H, T, 1.0 / math.sqrt(dk), p, seed, 11)
    f32 = dict(math="f32")
    dPd = torch.empty(B, H, T, T, device="cuda")
    K.gemm(do, qkv[:, 2 * d:], dPd, T, T, dk, d, 1, 1, 3 * d, T, 1, amode=_lib.LD_KC, bmode=_lib.LD_KC,
           batch=(B, H), bA=(T * d, dk), bB=(T * 3 * d, dk), bC=(H * T * T, T * T), **f32)
    dac = torch.empty(B, H, T, T, device="cuda")
    dbd = torch.empty(B, H, T, npos, device="cuda")
    K.relpos_softmax_bwd(P, dPd, dac, dbd, B, H, T, 1.0 / math.sqrt(dk), p, seed, 11)
    rows = B * T
    r_dv = torch.zeros(rows, d, device="cuda")
    K.gemm(Pd, do, r_dv, T, dk, T, 1, T, d, 1, d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * d, dk), bC=(T * d, dk), **f32)
    r_dqu = torch.zeros(rows, d, device="cuda")
    K.gemm(dac, qkv[:, d:], r_dqu, T, dk, T, T, 1, 3 * d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * 3 * d, dk), bC=(T * d, dk), **f32)
    r_dk = torch.zeros(rows, d, device="cuda")
    K.gemm(dac, qu, r_dk, T, dk, T, 1, T, d, 1, d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * T, T * T), bB=(T * d, dk), bC=(T * d, dk), **f32)
    r_dqv = torch.zeros(rows, d, device="cuda")
    K.gemm(dbd, ppos, r_dqv, T, dk, npos, npos, 1, d, 1, d, 1, amode=_lib.LD_KC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * npos, T * npos), bB=(0, dk), bC=(T * d, dk), **f32)
    r_dpos = torch.zeros(npos, d, device="cuda")
    K.gemm(dbd, qv, r_dpos, npos, dk, T, 1, npos, d, 1, d, 1, amode=_lib.LD_XC, bmode=_lib.LD_XC,
           batch=(B, H), bA=(H * T * npos, T * npos), bB=(T * d, dk), bC=(0, dk), epi=_lib.EPI_ATOMIC, **f32)
    torch.cuda.synchronize()
    return o, (r_dqu, r_dqv, r_dk, r_dv, r_dpos)


def test_attn_bwd_matches_unfused_with_dropout():
    from kdfm import kernels as K
    B, H, T, d, p = 2, 2, 401, 88, 0.1
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, 5)
    seed = torch.tensor([4242], dtype=torch.int64, device="cuda")
    _, o1, dqu, dqv, dk_, dv_, dpos = _fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    again = _fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    for a, b in zip((dqu, dqv, dk_, dv_, dpos), again[2:]):
        assert torch.equal(a, b), "fused attention backward is not bitwise reproducible"
    o, ref = _unfused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    # the single-pass output (online softmax, dropout on the unnormalised probabilities) = the two-pass one
    assert _rel(o1, o) <= 1e-2, _rel(o1, o)
    for name, got, want in zip(("dQu", "dQv", "dK", "dV", "dPpos"), (dqu, dqv, dk_, dv_, dpos), ref):
        assert _rel(got, want) <= 2e-2, (name, _rel(got, want))


def test_attn_bwd_parts_on_two_streams_match_one_launch():
    """kdfm_relpos_attn_bwd_parts: ROWDOT | DQ | DKV on one stream and DPOS (+ fold) on a second stream
    ordered after it (the engine puts DPOS on the weight-gradient stream) give bitwise the outputs of
    the single-stream call."""
    from kdfm import kernels as K
    B, H, T, d, p = 4, 2, 101, 88, 0.1
    dk = d // H
    seed = torch.tensor([77], dtype=torch.int64, device="cuda")
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, 3)
    ref = _fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    (lse, pt, mblk), o = ref[0], ref[1]
    dqu = torch.empty(B * T, d, device="cuda")
    dqv = torch.empty_like(dqu)
    dqkv = torch.zeros(B * T, 3 * d, device="cuda")
    dpos = torch.empty(2 * T - 1, d, device="cuda")
    ws = torch.empty(K.relpos_attn_bwd_ws(B, H, T, d), device="cuda")
    sc = 1.0 / math.sqrt(dk)
    K.relpos_attn_bwd(do, o, qu, qv, qkv, ppos, lse, pt, mblk, lens, dqu, dqv, dqkv, None, B, H, T, sc, p, seed, 11,
                      parts=K.ATTN_BWD_ROWDOT | K.ATTN_BWD_DQ | K.ATTN_BWD_DKV, ws=ws)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        K.relpos_attn_bwd(do, o, qu, qv, qkv, ppos, lse, pt, mblk, lens, None, None, None, dpos, B, H, T, sc, p, seed, 11,
                          parts=K.ATTN_BWD_DPOS, ws=ws)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for got, want in zip((dqu, dqv, dqkv[:, d:2 * d], dqkv[:, 2 * d:], dpos), ref[2:]):
        assert torch.equal(got, want)


def _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed, two_streams=False):
    """bwd2: lse-only single-pass forward, then _dq (writes the bf16 dS / Pd), _dkv and _dpos (optionally
    on a second stream, as the engine runs it); returns (O, lse, dS, Pd, grads...)."""
    dk = d // H
    lse = torch.empty(B, H, T, device="cuda")
    o = torch.empty(B * T, d, device="cuda")
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o, None, None, B, H, T, 1.0 / math.sqrt(dk), p, seed, 11, lse=lse)
    dqu = torch.empty(B * T, d, device="cuda")
    dqv = torch.empty_like(dqu)
    dqkv = torch.zeros(B * T, 3 * d, device="cuda")
    dpos = torch.empty(2 * T - 1, d, device="cuda")
    rsum = torch.empty(B * H * T, device="cuda")
    dS, Pd = K.attn_bwd2_saved(B, H, T, "cuda")
    K.relpos_attn_bwd2_dq(do, o, qu, qv, qkv, ppos, lse, lens, rsum, dS, Pd, dqu, dqv, B, H, T, 1.0 / math.sqrt(dk), p,
                          seed, 11)
    if two_streams:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            K.relpos_attn_bwd2_dpos(qv, dS, lens, dpos, B, H, T)
    else:
        K.relpos_attn_bwd2_dpos(qv, dS, lens, dpos, B, H, T)
    K.relpos_attn_bwd2_dkv(do, qu, dS, Pd, lens, dqkv, B, H, T)
    if two_streams:
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    return o, lse, dS, Pd, dqu, dqv, dqkv[:, d:2 * d], dqkv[:, 2 * d:], dpos


@pytest.mark.parametrize("B,H,T,d", [(3, 2, 401, 88), (2, 4, 130, 176), (2, 2, 77, 88), (2, 8, 201, 512),
                                     (2, 2, 77, 128)])
def test_attn_bwd2_matches_float64(B, H, T, d):
    """bwd2 (the dQ kernel saves bf16 dS and Pd; dK / dV / dPpos are plain products over them) against
    float64 autograd: rel. Frobenius <= 2e-2 per gradient; the saved Pd equals the float64 P on every
    valid (query, key) (no dropout: max |diff| <= 1e-2 max P + 1e-3); keys past a length get exactly zero
    dK / dV."""
    from kdfm import kernels as K
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, T + d + 1)
    seed = torch.tensor([98], dtype=torch.int64, device="cuda")
    _, _, dS, Pd, dqu, dqv, dk_, dv_, dpos = _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, 0.0, seed)
    ref = _torch_grads(qkv, qu, qv, ppos, do, lens, B, H, T, d)
    for name, got, want in zip(("dQu", "dQv", "dK", "dV", "dPpos"), (dqu, dqv, dk_, dv_, dpos), ref):
        assert _rel(got, want) <= 2e-2, (name, _rel(got, want))
    for bi in range(B):
        L = int(lens[bi])
        pw = _torch_grads.P[bi, :, :L, :L]
        perr = (Pd[bi, :, :L, :L].double() - pw).abs().max().item()
        assert perr <= 1e-2 * pw.abs().max().item() + 1e-3, (bi, perr)
        if L < T:
            assert dk_.view(B, T, d)[bi, L:].abs().max().item() == 0.0
            assert dv_.view(B, T, d)[bi, L:].abs().max().item() == 0.0


def test_attn_bwd2_matches_bwd1_with_dropout():
    """With attention dropout 0.1 the bwd2 gradients equal the recompute backward's (same counter-RNG mask)
    to bf16 level (rel. Frobenius <= 1e-2), the saved Pd is exactly 0 where the mask drops a valid
    probability and P / (1 - p) elsewhere (the recompute path's P to bf16 precision), dPpos on a second
    stream is bitwise the one-stream result, and two runs are bitwise identical."""
    from kdfm import kernels as K
    B, H, T, d, p = 3, 2, 401, 88, 0.1
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, 6)
    seed = torch.tensor([4243], dtype=torch.int64, device="cuda")
    one = _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    two = _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed, two_streams=True)
    for a, b in zip(one[4:], two[4:]):
        assert torch.equal(a, b), "bwd2 is not bitwise reproducible / stream-order independent"
    (lse1, pt, mblk), o1, *g1 = _fused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    for name, got, want in zip(("dQu", "dQv", "dK", "dV", "dPpos"), one[4:], g1):
        assert _rel(got, want) <= 1e-2, (name, _rel(got, want))
    assert torch.equal(one[0], o1) and torch.equal(one[1], lse1)
    Pd = one[3]
    for bi in range(B):
        L = int(lens[bi])
        kb = torch.arange(L, device="cuda") // 64
        prec = pt[bi, :, :L, :L].float() * torch.exp(mblk[bi, :, :L][:, :, kb] - lse1[bi, :, :L, None])
        got = Pd[bi, :, :L, :L].float()
        dropped = got == 0
        frac = (dropped & (prec > 1e-20)).double().sum().item() / max(1.0, (prec > 1e-20).double().sum().item())
        assert 0.07 < frac < 0.13, frac
        kept = ~dropped
        err = (got[kept] - prec[kept] / (1 - p)).abs().max().item()
        assert err <= 2e-2 * (prec.max().item() / (1 - p)) + 1e-3, (bi, err)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_bwd2_common_mode_keys_values(p):
    """Keys and values sharing a per-channel offset (3x their spread: the FastConformer layer-0 keys carry
    one, tools/attn_small_diag.py) -- the forward centres K and V on the utterance's first row before their
    bf16 rounding and the backward adds c_i = dO_i . v0 back in f32, so the offset costs no accuracy: the
    output and every bwd2 gradient within rel. Frobenius 2e-2 of float64 autograd (no dropout) or of the
    unfused f32 chain (dropout 0.1, same mask).  Uncentred, dQu was 6-10 % off here."""
    from kdfm import kernels as K
    B, H, T, d = 2, 8, 201, 512
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, 31)
    g = torch.Generator(device="cuda").manual_seed(1)
    qkv[:, d:] += 3.0 * torch.randn(1, 2 * d, device="cuda", generator=g)
    seed = torch.tensor([77], dtype=torch.int64, device="cuda")
    o, _, _, _, *got = _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    if p == 0.0:
        ref = _torch_grads(qkv, qu, qv, ppos, do, lens, B, H, T, d)
    else:
        o_ref, ref = _unfused(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
        assert _rel(o, o_ref) <= 1e-2, _rel(o, o_ref)
    for name, a, w in zip(("dQu", "dQv", "dK", "dV", "dPpos"), got, ref):
        assert _rel(a, w) <= 2e-2, (name, _rel(a, w))


def _torch_o_grads_masked(qkv, qu, qv, ppos, do, lens, B, H, T, d, keep, p):
    """float64 autograd of the attention with a given dropout keep mask (B, H, T, T) applied to P
    (Pd = P * keep / (1 - p)): O and the five input gradients."""
    dk = d // H
    f = lambda t: t.double().detach().clone().requires_grad_(True)  # noqa: E731
    q_u, q_v, k, v, pp = f(qu), f(qv), f(qkv[:, d:2 * d]), f(qkv[:, 2 * d:]), f(ppos)
    sh = lambda t: t.view(B, T, H, dk).permute(0, 2, 1, 3)  # noqa: E731
    ac = sh(q_u) @ sh(k).transpose(-1, -2)
    bdf = torch.einsum("bhic,hrc->bhir", sh(q_v), pp.view(2 * T - 1, H, dk).permute(1, 0, 2))
    idx = (T - 1 - torch.arange(T, device="cuda")[:, None] + torch.arange(T, device="cuda")[None, :])
    bd = torch.gather(bdf, 3, idx.expand(B, H, T, T))
    s = (ac + bd) / math.sqrt(dk)
    keym = torch.arange(T, device="cuda")[None, :] < lens[:, None]
    s = s.masked_fill(~keym[:, None, None, :], float("-inf"))
    P = torch.softmax(s, -1)
    P = torch.where(keym[:, None, :, None], P, torch.zeros_like(P))
    if keep is not None:
        P = P * keep.double() / (1.0 - p)
    O = (P @ sh(v)).permute(0, 2, 1, 3).reshape(B * T, d)
    loss = (O * do.double()).sum()
    return O.detach(), torch.autograd.grad(loss, [q_u, q_v, k, v, pp])


@pytest.mark.parametrize("B,H,T,d,p,kcm", [
    # FastConformer-XL (fast-conformer_ctc_bpe.yaml:29: d_model 1024, 8 heads -> head dim 128)
    (2, 8, 201, 1024, 0.0, 0.0),
    (2, 8, 201, 1024, 0.1, 0.0),
    (2, 8, 130, 1024, 0.0, 3.0),   # keys / values with a shared per-channel offset (attn_centre.h)
    (3, 1, 401, 128, 0.0, 0.0),    # one head, the benchmark's 401 frames, ragged lengths
    (2, 2, 77, 192, 0.1, 0.0),     # head dim 96: padded to the 128-wide kernels
    (1, 1, 65, 100, 0.0, 0.0),     # head dim 100 (not a multiple of 16)
])
def test_attn_head_dim_128_matches_float64(B, H, T, d, p, kcm):
    """Head dims 65..128 (the NU = 8 / 4-k-step instances of the single-pass forward and the bwd2 backward;
    the engine's route for FastConformer-XL): O and every gradient against float64 autograd, rel. Frobenius
    <= 2e-2 (bf16 operands, f32 accumulation).  With attention dropout the float64 reference applies the
    kernel's own keep mask (read back from the saved Pd: zero exactly where a valid probability was dropped),
    and the dropped fraction is checked against p; keys past a length get exactly zero dK / dV; the bwd2
    kernels are bitwise reproducible and dPpos on a second stream equals the one-stream result."""
    from kdfm import kernels as K
    qkv, qu, qv, ppos, do, lens = _inputs(B, H, T, d, 7 * T + d)
    if kcm:
        g = torch.Generator(device="cuda").manual_seed(2)
        qkv[:, d:] += kcm * torch.randn(1, 2 * d, device="cuda", generator=g)
    seed = torch.tensor([4099], dtype=torch.int64, device="cuda")
    one = _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed)
    two = _bwd2(K, qkv, qu, qv, ppos, do, lens, B, H, T, d, p, seed, two_streams=True)
    for i, (a, b) in enumerate(zip(one, two)):
        if i in (2, 3):   # dS / Pd: each utterance's valid (query, key) square (the rest is never written or read)
            for bi in range(B):
                L = int(lens[bi])
                assert torch.equal(a[bi, :, :L, :L], b[bi, :, :L, :L]), ("not bitwise reproducible", i, bi)
            continue
        assert torch.equal(a, b), ("not bitwise reproducible / stream-order independent", i)
    o, lse, dS, Pd, *got = one
    Pd = Pd[..., :T].clone()
    for bi in range(B):   # outside the valid square: unwritten
        L = int(lens[bi])
        Pd[bi, :, L:] = 0
        Pd[bi, :, :, L:] = 0
    keep = None
    if p > 0:
        valid = (torch.arange(T, device="cuda")[None, :] < lens[:, None])
        vq = valid[:, None, :, None] & valid[:, None, None, :]
        keep = (Pd.float() != 0) | ~vq
        dropped = (~keep & vq).double().sum().item() / vq.double().sum().item() / H
        assert 0.07 < dropped < 0.13, dropped
    o_ref, ref = _torch_o_grads_masked(qkv, qu, qv, ppos, do, lens, B, H, T, d, keep, p)
    valid_rows = (torch.arange(T, device="cuda")[None, :] < lens[:, None]).reshape(-1)
    assert _rel(o[valid_rows], o_ref[valid_rows]) <= 2e-2, ("O", _rel(o[valid_rows], o_ref[valid_rows]))
    for name, a, w in zip(("dQu", "dQv", "dK", "dV", "dPpos"), got, ref):
        assert _rel(a, w) <= 2e-2, (name, _rel(a, w))
    dk_, dv_ = got[2], got[3]
    for bi in range(B):
        L = int(lens[bi])
        if L < T:
            assert dk_.view(B, T, d)[bi, L:].abs().max().item() == 0.0
            assert dv_.view(B, T, d)[bi, L:].abs().max().item() == 0.0
