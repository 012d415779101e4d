"""The prepared-operand attention forward (kdfm_relpos_attn_fwd3, csrc/attn_fwd3.hip: bf16 centred K / V tiles
and positional band rows staged by LDS-DMA, rel_shift by lane permutes, the softmax in the exp2 domain with per-lane
partial row sums, dropout pair hashes shared between neighbouring lanes) against the register-staged single-pass
forward (kdfm_relpos_attn_fwd) it replaces on the bwd2 / inference path: the same bf16 operands and MFMAs and the
same dropout mask (common.h attn_drop_keep), so O and lse agree to f32 rounding of the softmax (a bf16 rounding of
a probability may flip: O within 1e-3, lse within 2e-6 relative) -- at the student / teacher / FastConformer / XL
head dims, ragged lengths, with attention dropout, and without lse (inference); the batched band preparation of
several layers equals the per-layer one; the prepared images hold exactly bf16(K - kc) / bf16(V - vc) with zero
padding."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(B, H, T, d, seed, kcm=0.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rows = B * T
    qkv = torch.randn(rows, 3 * d, device="cuda", generator=g)
    if kcm:
        qkv[:, d:] += kcm * torch.randn(1, 2 * d, device="cuda", generator=g)
    qu = torch.randn(rows, d, device="cuda", generator=g)
    qv = torch.randn(rows, d, device="cuda", generator=g)
    ppos = torch.randn(2 * T - 1, d, device="cuda", generator=g)
    lens = torch.tensor([T] + [max(1, T - 37 * (i + 1)) for i in range(B - 1)], dtype=torch.int64, device="cuda")
    return qkv, qu, qv, ppos, lens


@pytest.mark.parametrize("B,H,T,d,p,with_lse", [
    (4, 2, 401, 88, 0.1, True),     # the student (d88 / 2 heads, head dim 44), bench frames
    (3, 4, 401, 176, 0.0, False),   # the teacher (inference: no lse)
    (2, 8, 201, 512, 0.1, True),    # FastConformer d512 / 8 heads (head dim 64)
    (2, 8, 130, 1024, 0.1, True),   # FastConformer-XL (head dim 128)
    (3, 2, 77, 88, 0.0, True),      # T not a multiple of 64, short utterances
    (2, 1, 65, 100, 0.0, True),     # head dim 100
])
def test_fwd3_matches_register_staged(B, H, T, d, p, with_lse):
    from kdfm import kernels as K
    qkv, qu, qv, ppos, lens = _inputs(B, H, T, d, 5 * T + d, kcm=2.0)
    seed = torch.tensor([321], dtype=torch.int64, device="cuda")
    sc = 1.0 / math.sqrt(d // H)
    o1 = torch.empty(B * T, d, device="cuda")
    lse1 = torch.empty(B, H, T, device="cuda") if with_lse else None
    K.relpos_attn_fwd(qu, qv, qkv, ppos, lens, o1, None, None, B, H, T, sc, p, seed, 17, lse=lse1)
    o2 = torch.full((B * T, d), float("nan"), device="cuda")
    lse2 = torch.full((B, H, T), float("nan"), device="cuda") if with_lse else None
    prep = K.attn_kv_prep(qkv, lens, B, H, T)
    pb = K.attn_band_prep(ppos, H, T)[0]
    K.relpos_attn_fwd3(qu, qv, prep, pb, lens, o2, B, H, T, sc, p, seed, 17, lse=lse2)
    torch.cuda.synchronize()
    assert not torch.isnan(o2).any()
    torch.testing.assert_close(o2, o1, rtol=1e-3, atol=1e-3)
    if with_lse:
        torch.testing.assert_close(lse2, lse1, rtol=2e-6, atol=2e-6)


def test_prepared_images_and_batched_band():
    from kdfm import kernels as K
    B, H, T, d = 2, 2, 77, 88
    dk = d // H
    qkv, qu, qv, ppos, lens = _inputs(B, H, T, d, 9, kcm=1.0)
    kb, vb, cen = K.attn_kv_prep(qkv, lens, B, H, T)
    Tp, LR = 128, 56   # head dim 44 -> padded to 48 (attn_prep_dkp) + 8
    kb = kb.view(B, H, Tp, LR).float().cpu()
    vb = vb.view(B, H, Tp, LR).float().cpu()
    cen = cen.view(B, H, 2, 48).cpu()
    x = qkv.view(B, T, 3, H, dk).cpu()
    for b in range(B):
        n = min(16, int(lens[b]))
        n = 1 << (n.bit_length() - 1)
        for h in range(H):
            for kind, img in ((1, kb), (2, vb)):
                c = x[b, :n, kind, h].sum(0) / n   # in-order f32 sum of the first n rows (attn_centre.h)
                assert torch.allclose(cen[b, h, kind - 1, :dk], c, rtol=0, atol=1e-6)
                want = (x[b, :, kind, h] - cen[b, h, kind - 1, :dk]).bfloat16().float()
                assert torch.equal(img[b, h, :T, :dk], want)
                assert img[b, h, T:].abs().max() == 0 and img[b, h, :, dk:].abs().max() == 0
    # three layers' projections in one launch == one launch per layer
    g = torch.Generator(device="cuda").manual_seed(3)
    pp = torch.randn(3, 2 * T - 1, d, device="cuda", generator=g)
    allb = K.attn_band_prep(pp, H, T)
    for l in range(3):
        assert torch.equal(allb[l], K.attn_band_prep(pp[l], H, T)[0])
    band = allb[1].view(H, 64 + 2 * T - 1 + 88, LR).float().cpu()
    want = pp[1].view(2 * T - 1, H, dk).permute(1, 0, 2).bfloat16().float().cpu()
    assert torch.equal(band[:, 64:64 + 2 * T - 1, :dk], want)
    assert band[:, :64].abs().max() == 0 and band[:, 64 + 2 * T - 1:].abs().max() == 0 and band[:, :, dk:].abs().max() == 0


@pytest.mark.parametrize("B,H,T,d,p", [(4, 2, 401, 88, 0.1), (2, 8, 201, 512, 0.0), (2, 8, 130, 1024, 0.1),
                                       (3, 2, 77, 88, 0.0)])
def test_dq3_equals_register_staged_dq(B, H, T, d, p):
    """The bwd2 dQ kernel over the forward's prepared operands (kdfm_relpos_attn_bwd2_dq3) against the one that
    stages K / V / the band from qkv / pos: the same bf16 operands and dropout mask; at head dims <= 48 the
    prepared tiles are padded to 48 (a 32- and a 16-wide MFMA k-step) where the staged ones pad to 64, so the
    scores differ by f32 summation order only: dS / Pd within a bf16 rounding (2^-7 relative + 1e-6),
    dqu / dqv within 1e-3 relative Frobenius; bitwise at the other head dims."""
    from kdfm import kernels as K
    qkv, qu, qv, ppos, lens = _inputs(B, H, T, d, 3 * T + d, kcm=1.5)
    g = torch.Generator(device="cuda").manual_seed(T)
    do = torch.randn(B * T, d, device="cuda", generator=g)
    seed = torch.tensor([99], dtype=torch.int64, device="cuda")
    sc = 1.0 / math.sqrt(d // H)
    o = torch.empty(B * T, d, device="cuda")
    lse = torch.empty(B, H, T, device="cuda")
    prep = K.attn_kv_prep(qkv, lens, B, H, T)
    pb = K.attn_band_prep(ppos, H, T)[0]
    K.relpos_attn_fwd3(qu, qv, prep, pb, lens, o, B, H, T, sc, p, seed, 5, lse=lse)
    outs = []
    for dq3 in (False, True):
        dS, Pd = K.attn_bwd2_saved(B, H, T, "cuda")
        dS.fill_(0)
        Pd.fill_(0)
        dqu = torch.empty(B * T, d, device="cuda")
        dqv = torch.empty(B * T, d, device="cuda")
        if dq3:
            K.relpos_attn_bwd2_dq3(do, o, qu, qv, prep, pb, lse, lens, dS, Pd, dqu, dqv, B, H, T, sc, p, seed, 5)
        else:
            K.relpos_attn_bwd2_dq(do, o, qu, qv, qkv, ppos, lse, lens, None, dS, Pd, dqu, dqv, B, H, T, sc, p, seed, 5)
        outs.append((dS, Pd, dqu, dqv))
    torch.cuda.synchronize()
    (a0, b0, c0, e0), (a1, b1, c1, e1) = outs
    if d // H > 48:
        assert torch.equal(a0, a1) and torch.equal(b0, b1)
        assert (c0 - c1).abs().max().item() == 0.0 and (e0 - e1).abs().max().item() == 0.0
        return
    for x, y in ((a0, a1), (b0, b1)):
        x, y = x.float(), y.float()
        assert ((x - y).abs() <= y.abs() * 2.0 ** -7 + 1e-6).all(), (x - y).abs().max().item()
    for x, y in ((c0, c1), (e0, e1)):
        assert ((x - y).norm() / y.norm()).item() <= 1e-3
