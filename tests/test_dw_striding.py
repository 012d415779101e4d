"""'dw_striding' subsampling (north_star: "depthwise-separable conv subsampling"; built at
NeMo/nemo/collections/asr/modules/conformer_encoder.py:381-390, recipe
NeMo/examples/asr/conf/fastconformer/fast-conformer_ctc_bpe.yaml:122-125) — CPU checks of the oracle
restatement (oracle/ver5.py subsampling_dw_striding; the module source is absent, SURVEY.md
Appendix A) and of the host-side naming / shape logic the HIP path uses.

Pinned by NeMo/tests/collections/asr/test_padding_and_batch_size_invariance.py:49-130: the
subsampling output (and every inner conv output) on the valid frames is unchanged when the input
is right-padded with zeros and the lengths are kept.  Absolute values are "parity unpinned" (no
reference fixture exists for this module); the GPU path is pinned to this oracle by
tests/test_dw_striding_gpu.py.
"""
from dataclasses import replace

import pytest
import torch

from oracle import ver5


def _cfg(factor, causal, C=32):
    return replace(ver5.StepConfig(), subsampling="dw_striding", subsampling_factor=factor,
                   subsampling_conv_channels=C, causal_downsampling=causal)


def _params(cfg, d, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {k: (torch.rand(s, generator=g, dtype=torch.float64) * 2 - 1) * 0.3
            for k, s in ver5.subsampling_param_shapes(cfg, d).items()}


@pytest.mark.parametrize("factor,causal", [(4, False), (8, False), (8, True), (16, False)])
def test_dw_striding_invariant_to_right_padding(factor, causal):
    cfg = _cfg(factor, causal)
    d = 48
    p = _params(cfg, d)
    g = torch.Generator().manual_seed(1)
    T = 101                                   # 1 s of 10 ms frames (the reference test's 16000 samples)
    x1 = torch.randn(1, T, cfg.nfilt, generator=g, dtype=torch.float64)
    x2 = torch.cat([x1, torch.zeros(1, 100, cfg.nfilt, dtype=torch.float64)], dim=1)
    L = torch.tensor([T])
    h1, l1 = ver5.subsampling(x1, L, p, "pre_encode.", cfg)
    h2, l2 = ver5.subsampling(x2, L, p, "pre_encode.", cfg)
    assert int(l1) == int(l2)
    n = int(l1)
    torch.testing.assert_close(h1[:, :n], h2[:, :n], rtol=0, atol=1e-12)


def test_without_the_mask_padding_leaks():
    """The masks are what makes it invariant (a right-padded batch row differs without them)."""
    cfg = replace(_cfg(8, True), subsampling_mask=False)
    p = _params(cfg, 48)
    x1 = torch.randn(1, 101, cfg.nfilt, dtype=torch.float64) + 3.0
    x2 = torch.cat([x1, torch.full((1, 100, cfg.nfilt), 3.0, dtype=torch.float64)], dim=1)
    L = torch.tensor([101])
    h1, l1 = ver5.subsampling(x1, L, p, "pre_encode.", cfg)
    h2, _ = ver5.subsampling(x2, L, p, "pre_encode.", cfg)
    n = int(l1)
    assert not torch.allclose(h1[:, :n], h2[:, :n], atol=1e-6)


@pytest.mark.parametrize("factor,causal,T,want", [
    (8, True, 101, [51, 26, 14]),        # CausalConv2D: floor(l / 2) + 1 per stage
    (8, False, 101, [51, 26, 13]),       # symmetric: floor((l - 1) / 2) + 1
    (8, False, 1601, [801, 401, 201]),   # 16 s FastConformer frames
    (4, False, 1601, [801, 401]),
])
def test_stage_lengths(factor, causal, T, want):
    cfg = _cfg(factor, causal)
    L = torch.tensor([T])
    got = []
    for _ in range(len(want)):
        L = ver5.sub_stage_len(L, cfg)
        got.append(int(L))
    assert got == want
    x = torch.zeros(1, T, cfg.nfilt, dtype=torch.float64)
    h, n = ver5.subsampling(x, torch.tensor([T]), _params(cfg, 16), "pre_encode.", cfg)
    assert h.shape[1] == want[-1] == int(n)


def test_zero_length_rows_stay_zero():
    cfg = _cfg(8, False)
    p = _params(cfg, 16)
    x = torch.randn(2, 60, cfg.nfilt, dtype=torch.float64)
    h, n = ver5.subsampling(x, torch.tensor([60, 0]), p, "pre_encode.", cfg)
    assert int(n[1]) == 0
    # every frame of the empty row is the output Linear's bias alone
    torch.testing.assert_close(h[1], p["pre_encode.out.bias"].expand_as(h[1]))


def test_module_names_and_shapes_match_the_nemo_sequential():
    """conv.0 = Conv2d(1, C), conv.1 ReLU, then per stage conv.{i} depthwise (C, 1, 3, 3),
    conv.{i+1} pointwise (C, C, 1, 1), conv.{i+2} ReLU; out = Linear(C * F', d); the engine's
    flat-buffer specs (kdfm.config.subsampling_specs) carry the same names and shapes."""
    from kdfm.config import Ver5Config, sub_dims, subsampling_specs
    for factor, causal, C in [(8, False, 256), (8, True, 64), (4, False, 88), (16, True, 32)]:
        ocfg = _cfg(factor, causal, C)
        kcfg = Ver5Config(subsampling="dw_striding", subsampling_factor=factor, subsampling_conv_channels=C,
                          causal_downsampling=causal)
        want = ver5.subsampling_param_shapes(ocfg, 176)
        got = dict(subsampling_specs(kcfg, 176, ""))
        assert got == want
        Fo = sub_dims(kcfg, 1601)[-1][1]
        assert want["pre_encode.out.weight"] == (176, C * Fo) == (176, C * ver5.sub_out_features(ocfg))
    names = list(ver5.subsampling_param_shapes(_cfg(8, False, 256), 512))
    assert names == ["pre_encode.conv.0.weight", "pre_encode.conv.0.bias",
                     "pre_encode.conv.2.weight", "pre_encode.conv.2.bias",
                     "pre_encode.conv.3.weight", "pre_encode.conv.3.bias",
                     "pre_encode.conv.5.weight", "pre_encode.conv.5.bias",
                     "pre_encode.conv.6.weight", "pre_encode.conv.6.bias",
                     "pre_encode.out.weight", "pre_encode.out.bias"]
    # FastConformer recipe: 80 mel features -> 10 after x8, Linear(256 * 10 -> 512)
    assert ver5.subsampling_param_shapes(_cfg(8, False, 256), 512)["pre_encode.out.weight"] == (512, 2560)
