"""'dw_striding' subsampling on the GPU (csrc/dwsub.hip + kdfm_gemm), through the NeMo module API
(kdfm.nemo.ConvSubsampling / ConformerEncoder, conformer_encoder.py:381-390).

1. Module forward + backward against the oracle restatement (oracle/ver5.py
   subsampling_dw_striding) evaluated in float64 with torch autograd, ragged lengths (one row
   shorter than the first stride), factors x4 / x8 / x16, symmetric and causal padding.
   Tolerances: f32 parity mode — output and every parameter gradient max|diff| <= 1e-4 * max|ref|
   (+1e-6); bf16 MFMA mode (pointwise convs and the output Linear in bf16 operands, f32
   accumulation) — output relative Frobenius error <= 3e-2; each gradient's relative Frobenius
   error <= max(3e-2, 2.5 x the oracle's own sensitivity to bf16 rounding), where the sensitivity
   is measured by re-running the float64 oracle with only the GEMM weights rounded to bf16: with
   random weights many ReLU pre-activations sit near zero, a rounding flips their mask, and the
   early layers' gradients move ~5% from that alone (measured 4.9% for conv.0.weight).
2. The reference's padding-invariance test (NeMo/tests/collections/asr/
   test_padding_and_batch_size_invariance.py:49-130, scaled down: 2 layers, d=96, 64 subsampling
   channels, causal x8, conv kernel 9, xscaling off, eval mode): 1 s of audio vs the same audio plus
   1 s of zeros with unchanged lengths -> equal mel on the valid frames (atol 5e-4), equal
   pre_encode output and equal encoder output on the valid frames (assert_close defaults).
"""
from dataclasses import replace

import pytest
import torch

from oracle import ver5 as O

pytestmark = pytest.mark.gpu


def _mod(factor, causal, C, d, math):
    from kdfm.config import Ver5Config
    from kdfm.nemo import ConvSubsampling
    cfg = Ver5Config(subsampling="dw_striding", subsampling_factor=factor, subsampling_conv_channels=C,
                     causal_downsampling=causal, xscaling=False, dropout_pre=0.0, math=math)
    m = ConvSubsampling(cfg, d, device="cuda")
    g = torch.Generator().manual_seed(factor * 10 + int(causal))
    with torch.no_grad():
        for name, prm in m.named_parameters():
            prm.copy_(((torch.rand(prm.shape, generator=g) * 2 - 1) * 0.3).cuda())
    ocfg = replace(O.StepConfig(), subsampling="dw_striding", subsampling_factor=factor, subsampling_conv_channels=C,
                   causal_downsampling=causal)
    return m, ocfg


def _close(a, b, tol, what, rn=None):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= tol * scale + 1e-6, f"{what}: max|diff| {err:.3e} vs max|ref| {scale:.3e}"
    if rn is not None:
        r = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert r <= rn, f"{what}: relative Frobenius error {r:.3e}"


@pytest.mark.parametrize("factor,causal,C,math,tol,rn", [
    (4, False, 32, "f32", 1e-4, None),
    (8, False, 64, "f32", 1e-4, None),
    (8, True, 32, "f32", 1e-4, None),
    (16, True, 16, "f32", 1e-4, None),
    (8, False, 256, "f32", 1e-4, None),    # FastConformer's 256 channels (fast-conformer_ctc_bpe.yaml:122-125)
    (8, False, 64, "bf16", 1e-1, 3e-2),
])
def test_module_matches_oracle(factor, causal, C, math, tol, rn):
    from kdfm import kernels as K
    d = 48
    m, ocfg = _mod(factor, causal, C, d, math)
    g = torch.Generator().manual_seed(5)
    B, T = 3, 203
    x = torch.randn(B, T, 80, generator=g)
    lens = torch.tensor([T, 150, 1], dtype=torch.int64)
    with K.mode(math, True):
        xc = x.cuda()
        y, yl = m(xc, lens.cuda())
        R = torch.randn(y.shape, generator=g)
        (y * R.cuda()).sum().backward()
        torch.cuda.synchronize()
    p = {"pre_encode." + n: prm.detach().cpu().double().requires_grad_(True) for n, prm in m.named_parameters()}
    yo, lo = O.subsampling(x.double(), lens, p, "pre_encode.", ocfg)
    assert torch.equal(yl.cpu(), lo)
    _close(y, yo, tol, f"output ({math})", rn)
    go = torch.autograd.grad((yo * R.double()).sum(), list(p.values()))
    sens = {}
    if math == "bf16":
        gemm_w = [k for k in p if k.endswith("weight") and (k.startswith("pre_encode.out") or p[k].shape[-1] == 1)]
        pb = {k: (v.detach().bfloat16().double() if k in gemm_w else v.detach()).requires_grad_(True)
              for k, v in p.items()}
        yb, _ = O.subsampling(x.double(), lens, pb, "pre_encode.", ocfg)
        gb = torch.autograd.grad((yb * R.double()).sum(), list(pb.values()))
        sens = {k: ((b - a).norm() / a.norm().clamp_min(1e-30)).item() for k, a, b in zip(p, go, gb)}
    for (n, prm), gr in zip(m.named_parameters(), go):
        r = None if rn is None else max(rn, 2.5 * sens["pre_encode." + n])
        _close(prm.grad, gr, 1.0 if rn else tol, f"grad {n} ({math})", r)


def test_encoder_invariant_to_padding():
    """NeMo test_canary_encoder_invariant_to_padding, scaled down (see module docstring)."""
    from kdfm import kernels as K
    from kdfm.nemo import AudioToMelSpectrogramPreprocessor, ConformerEncoder
    with K.mode("f32", True):
        pre = AudioToMelSpectrogramPreprocessor(features=80).cuda().eval()
        enc = ConformerEncoder(feat_in=80, n_layers=2, d_model=96, n_heads=2, subsampling="dw_striding",
                               subsampling_factor=8, subsampling_conv_channels=64, causal_downsampling=True,
                               conv_kernel_size=9, xscaling=False, device="cuda").eval()
        length = 16000
        a1 = (torch.arange(0, length).unsqueeze(0) / 16000).cuda()
        a1l = torch.tensor([length]).cuda()
        a2 = torch.cat([a1, torch.zeros(1, 16000, device="cuda")], dim=1)
        mels1, mels1l = pre(input_signal=a1, length=a1l)
        mels2, _ = pre(input_signal=a2, length=a1l.clone())
        n = int(mels1l)
        torch.testing.assert_close(mels1[..., :n], mels2[..., :n], atol=5e-4, rtol=0)
        with torch.no_grad():
            h1, h1l = enc.pre_encode(mels1.transpose(1, 2), mels1l)
            h2, h2l = enc.pre_encode(mels2.transpose(1, 2), mels1l)
            assert int(h1l) == int(h2l) == 14   # 101 mel frames -> 51 -> 26 -> 14 (causal)
            k = int(h1l)
            torch.testing.assert_close(h1[:, :k], h2[:, :k])
            e1, e1l = enc(audio_signal=mels1, length=mels1l)
            e2, _ = enc(audio_signal=mels2, length=mels1l)
            torch.testing.assert_close(e1[..., :int(e1l)], e2[..., :int(e1l)])
