"""Training-mode randomness of the benchmarked step, all drawn on device from the counter RNG
(common.h rng_bits: splitmix64 over (seed, stream, index)), checked for the properties the
reference's draws have:

* SpecAugment (NeMo SpectrogramAugmentation, audio_preprocessing.py:443-553, called
  asr_train_diffm.py:622-623; recipe conformer_ctc_bpe.yaml:108-114:
  2 frequency masks of width <= 27, 5 time masks of width <= 0.05*len): with injected uniforms the
  masks equal the oracle's restatement of NeMo's vectorized form bit for bit; drawn on device, masked cells exactly 0,
  others untouched; the mask of an utterance is (frequency band set) x all frames  U  all bins x
  (time band set); at most 2 frequency runs (union width <= 54) and 5 time runs, time runs inside the
  valid length; mean widths match the uniform width draw; seeded (same seed -> same masks).
* dropout (p = 0.1, conformer_ctc_bpe.yaml:150-153): keep rate and 1/(1-p) scaling, and the GEMM
  epilogue's mask equals kdfm_dropout's for the same (seed, stream, index) — the backward regenerates
  the forward mask through the latter.
* NoiseAdapter eps (torch.randn_like, asr_train_diffm.py:438-441) generated on device: standard
  normal moments (mean, variance, kurtosis, tail mass) and no lag correlation.
* dither (FilterbankFeatures dither 1e-5, training only): dither*N(0,1) added before preemphasis,
  the same draw reused as x[n-1] of the next sample (lag-1 correlation -0.97/(1+0.97^2)), nothing
  past the utterance length.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _seed(v):
    return torch.tensor([v], dtype=torch.int64, device="cuda")


def _runs(mask_1d):
    m = mask_1d.to(torch.int8).tolist()
    runs, cur = [], 0
    for v in m + [0]:
        if v:
            cur += 1
        elif cur:
            runs.append(cur)
            cur = 0
    return runs


def test_specaugment_mask_structure():
    from kdfm import kernels as K
    B, T, nf = 48, 1601, 80
    g = torch.Generator().manual_seed(3)
    lens = torch.randint(700, T + 1, (B,), generator=g)
    lens[0] = T
    x0 = torch.randn(B, T, nf, generator=g).cuda()
    x = x0.clone()
    mask = torch.empty(B, T, nf, dtype=torch.uint8, device="cuda")
    K.specaugment(x, lens.cuda(), B, T, nf, 2, 27, 5, 0.05, _seed(99), 5, mask_out=mask)
    torch.cuda.synchronize()
    m = mask.bool().cpu()
    xc, x0c = x.cpu(), x0.cpu()
    assert torch.equal(xc[m], torch.zeros(int(m.sum())))
    assert torch.equal(xc[~m], x0c[~m])
    fw, tw = [], []
    for b in range(B):
        mb = m[b]
        tset = mb.all(dim=1)             # frames masked across all bins = time bands
        fset = mb.all(dim=0)             # bins masked across all frames = frequency bands
        assert torch.equal(mb, tset[:, None] | fset[None, :]), b
        fr, tr = _runs(fset), _runs(tset)
        assert len(fr) <= 2 and sum(fr) <= 54 and all(r <= 54 for r in fr), (b, fr)
        maxw = max(1, int(float(lens[b]) * 0.05))
        assert len(tr) <= 5 and all(r <= 5 * maxw for r in tr), (b, tr)
        if tset.any():
            assert int(tset.nonzero().max()) < int(lens[b]), b   # time masks stay inside the utterance
        fw.append(int(fset.sum()))
        tw.append(int(tset.sum()) / maxw)
    # uniform widths: E[w] = 13.5 per frequency mask (2 masks, overlaps shrink the union);
    # E[w] = maxw/2 per time mask (5 masks)
    assert 16.0 < sum(fw) / B < 30.0, sum(fw) / B
    assert 1.6 < sum(tw) / B < 2.9, sum(tw) / B
    # seeded: the same seed reproduces the masks, another seed does not
    m2 = torch.empty_like(mask)
    K.specaugment(x0.clone(), lens.cuda(), B, T, nf, 2, 27, 5, 0.05, _seed(99), 5, mask_out=m2)
    m3 = torch.empty_like(mask)
    K.specaugment(x0.clone(), lens.cuda(), B, T, nf, 2, 27, 5, 0.05, _seed(100), 5, mask_out=m3)
    assert torch.equal(m2, mask) and not torch.equal(m3, mask)


def test_specaugment_injected_uniforms_match_oracle():
    """Parity mode (RNG as an input): the kernel fed the same uniforms as the oracle's
    restatement of NeMo's vectorized SpecAugment (oracle.ver5.specaugment_mask, A.2: time width
    (int)(U min(0.05 len, T)), start (int)(U' (len - w)); freq width (int)(27 U), start (int)(U' (80 - w)))
    gives the IDENTICAL mask, at ragged lengths (incl. lengths where 0.05 len crosses an integer, len < 20,
    len = T) and edge uniforms (0, the largest float below 1, values landing on integer widths)."""
    from kdfm import kernels as K
    from oracle.ver5 import specaugment_mask
    B, T, nf, fm, tm = 40, 1601, 80, 2, 5
    g = torch.Generator().manual_seed(8)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    lens[:8] = torch.tensor([T, 1, 19, 20, 21, 39, 40, 1580])
    u = torch.rand(B, 2 * (fm + tm), generator=g)
    below1 = torch.nextafter(torch.tensor(1.0), torch.tensor(0.0))
    u[0] = below1
    u[1] = 0.0
    u[2, :tm] = 1.0 / (0.05 * 19)          # lands on width 1 before truncation
    u[3, 2 * tm:2 * tm + fm] = 1.0 / 27     # freq width exactly 1 in f32 or just below
    u[4, :] = below1
    u[5, tm:2 * tm] = below1                # starts at the last admissible frame
    x0 = torch.randn(B, T, nf, generator=g)
    x = x0.cuda()
    mask = torch.empty(B, T, nf, dtype=torch.uint8, device="cuda")
    K.specaugment(x, lens.cuda(), B, T, nf, fm, 27, tm, 0.05, None, 0, mask_out=mask, uniforms=u.cuda())
    torch.cuda.synchronize()
    want = specaugment_mask(lens, T, nf, u, fm, 27, tm, 0.05)
    got = mask.bool().cpu()
    bad = (got != want).nonzero()
    assert bad.numel() == 0, f"{bad.shape[0]} cells differ, first at (b, t, f) = {bad[0].tolist()}"
    assert want.any()
    xc = x.cpu()
    assert torch.equal(xc[want], torch.zeros(int(want.sum()))) and torch.equal(xc[~want], x0[~want])


def test_dropout_keep_rate_and_gemm_mask_agree():
    from kdfm import _lib
    from kdfm import kernels as K
    n = 1 << 21
    ones = torch.ones(n, device="cuda")
    out = torch.empty_like(ones)
    p = 0.1
    K.dropout(ones, out, p, 1.0, _seed(5), 41)
    o = out.cpu()
    keep = (o != 0).float().mean().item()
    assert abs(keep - (1 - p)) < 6 * math.sqrt(p * (1 - p) / n), keep
    assert torch.allclose(o[o != 0], torch.full_like(o[o != 0], 1 / (1 - p)))
    # GEMM epilogue dropout (the FFN / attention-out / conv-pw2 sites) vs the standalone kernel
    M, N = 4096, 96
    x = torch.randn(M, N, device="cuda")
    eye = torch.eye(N, device="cuda")
    y = torch.empty(M, N, device="cuda")
    with K.mode("f32"):
        K.linear(x, eye, None, y, dropout_p=p, seed=_seed(5), rng_stream=17)
    ref = torch.empty(M * N, device="cuda")
    K.dropout(torch.ones(M * N, device="cuda"), ref, p, 1.0, _seed(5), 17)
    assert torch.equal((y != 0).cpu(), (ref.view(M, N) != 0).cpu() & (x != 0).cpu())
    torch.testing.assert_close(y, x * ref.view(M, N), rtol=1e-6, atol=1e-6)
    assert _lib.EPI_DROPOUT


def test_noise_adapter_eps_is_standard_normal():
    from kdfm import kernels as K
    rows, L = 20000, 96
    zs = torch.zeros(rows, L, device="cuda")
    h = torch.zeros(rows, L, device="cuda")
    w2 = torch.zeros(L, device="cuda")
    b2 = torch.zeros(1, device="cuda")
    zn = torch.empty(rows, L, device="cuda")
    gam = torch.empty(rows, device="cuda")
    K.adapter_fwd(zs, h, w2, b2, None, zn, gam, _seed(123), 7)
    torch.cuda.synchronize()
    assert torch.all(gam == 0.5)
    e = (2.0 * zn).double().cpu().flatten()                # zn = 0.5*zs + 0.5*eps
    n = e.numel()
    mean, var = e.mean().item(), e.var().item()
    kurt = (((e - mean) ** 4).mean() / var ** 2).item()
    tail = (e.abs() > 2.0).double().mean().item()
    assert abs(mean) < 5 / math.sqrt(n), mean
    assert abs(var - 1.0) < 5 * math.sqrt(2.0 / n), var
    assert abs(kurt - 3.0) < 0.05, kurt
    assert abs(tail - 0.0455) < 0.002, tail
    lag = (e[1:] * e[:-1]).mean().item()
    assert abs(lag) < 5 / math.sqrt(n), lag
    # a different step seed gives different draws; the same seed the same draws
    zn2 = torch.empty_like(zn)
    K.adapter_fwd(zs, h, w2, b2, None, zn2, gam, _seed(123), 7)
    zn3 = torch.empty_like(zn)
    K.adapter_fwd(zs, h, w2, b2, None, zn3, gam, _seed(124), 7)
    assert torch.equal(zn, zn2) and not torch.equal(zn, zn3)


def test_dither_moments_and_preemphasis_coupling():
    from kdfm import kernels as K
    B, N, pad = 4, 160000, 256
    wav = torch.zeros(B, N, device="cuda")
    lens = torch.tensor([N, N, 120000, 80000], dtype=torch.int64, device="cuda")
    dither = 1e-5
    xp = torch.empty(B, N + 2 * pad, device="cuda")
    K.preemph_pad(wav, lens, xp, pad, 0.0, dither, _seed(8), 3)
    x = xp.double().cpu() / dither
    v = x[0, pad:pad + N]
    assert abs(v.mean().item()) < 5 / math.sqrt(N)
    assert abs(v.var().item() - 1.0) < 5 * math.sqrt(2.0 / N)
    assert torch.all(x[:, :pad] == 0) and torch.all(x[:, pad + N:] == 0)
    assert torch.all(x[2, pad + 120000:] == 0) and torch.all(x[3, pad + 80000:] == 0)
    # with preemphasis the same draw enters twice: y[n] = d*(e[n] - 0.97 e[n-1])
    K.preemph_pad(wav, lens, xp, pad, 0.97, dither, _seed(8), 3)
    y = xp.double().cpu()[0, pad + 1:pad + N] / dither
    e = v
    torch.testing.assert_close(y, e[1:] - 0.97 * e[:-1], rtol=1e-4, atol=1e-4)
    r1 = ((y[1:] * y[:-1]).mean() / y.var()).item()
    assert abs(r1 - (-0.97 / (1 + 0.97 ** 2))) < 0.02, r1
