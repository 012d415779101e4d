"""The step-parity carve-out for the subsampling's first conv (tests/test_step_parity_gpu.py first_conv_ok) is
bounded: the measured ReLU-flip case (profiles/r04/conv0_diag.log: one channel, 3.5e-3 of the tensor's max,
confined to taps 3-8) passes, while a 10 % corruption of any one channel's weight-gradient row, a corruption
of three channels, or an excepted row beyond 5e-3 of the tensor's max fails.  CPU only (pure tensor logic)."""
import torch

from test_step_parity_gpu import first_conv_ok

K_W = "encoder.pre_encode.conv.0.weight"
K_B = "encoder.pre_encode.conv.0.bias"


def _ref(seed=0, C=88):
    g = torch.Generator().manual_seed(seed)
    r = 0.3 * torch.randn(C, 1, 3, 3, generator=g, dtype=torch.float64)
    r[0, 0, 1, 1] = 0.881   # the tensor's max (the r04 log: 8.809e-01)
    r[54] *= 0.237 / r[54].abs().max()
    return r, g


def test_measured_flip_passes():
    r, g = _ref()
    mine = r + 1e-7 * torch.randn(r.shape, generator=g, dtype=torch.float64)
    # channel 54, taps 3-8: the per-tap errors of the overlapped run
    errs = torch.tensor([5.86e-04, 6.55e-04, 3.49e-03, 2.81e-03, 1.74e-03, 3.00e-04], dtype=torch.float64)
    mine[54].view(-1)[3:] += errs
    assert first_conv_ok(K_W, mine, r)
    b = 0.5 * torch.randn(88, generator=g, dtype=torch.float64)
    b[3] = 1.154
    mb = b.clone()
    mb[54] += 1.79e-3
    assert first_conv_ok(K_B, mb, b)


def test_other_tensors_never_excepted():
    r, _ = _ref()
    assert not first_conv_ok("encoder.pre_encode.conv.2.weight", r + 1e-3, r)


def test_ten_percent_one_channel_fails():
    r, _ = _ref()
    for c in (0, 17, 54, 87):
        mine = r.clone()
        mine[c] *= 1.10
        assert not first_conv_ok(K_W, mine, r), c


def test_three_channels_fail():
    r, _ = _ref()
    mine = r.clone()
    for c in (3, 9, 40):
        mine[c].view(-1)[5] += 3e-3
    assert not first_conv_ok(K_W, mine, r)


def test_unbounded_row_fails():
    r, _ = _ref()
    mine = r.clone()
    mine[54].view(-1)[5] += 1e-2   # 1.1 % of the tensor's max, 4 % of the row's: beyond 5e-3 x max
    assert not first_conv_ok(K_W, mine, r)
    b = torch.linspace(-1.0, 1.0, 88, dtype=torch.float64)
    mb = b.clone()
    mb[10] += 0.05
    assert not first_conv_ok(K_B, mb, b)
