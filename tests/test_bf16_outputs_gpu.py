"""bf16-output variants of the elementwise producers whose results only large-tile (bf16-operand) products read --
kdfm_dropout_bf16, kdfm_bn_silu_fwd_bf16, kdfm_glu_mask_bwd_bf16, kdfm_layernorm_fwd_bf16 (FastConformer(-XL) layers,
conformer.py _grad_bf16 / _ln_bf16): each must equal its f32 output rounded to nearest even, bit for bit -- the value
the large-tile route's own cast of the f32 output gave."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _K():
    from kdfm import kernels as K
    return K


def test_dropout_bf16_is_rounded_f32():
    K = _K()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(6432, 1024, device="cuda", generator=g)
    seed = torch.tensor([77], dtype=torch.int64, device="cuda")
    y = torch.empty_like(x)
    y16 = torch.empty(x.shape, device="cuda", dtype=torch.bfloat16)
    K.dropout(x, y, 0.1, 0.5, seed, 9)
    K.dropout(x, y16, 0.1, 0.5, seed, 9)
    torch.cuda.synchronize()
    assert torch.equal(y16, y.bfloat16())
    assert 0.09 < (y == 0).double().mean().item() < 0.11


def test_bn_silu_fwd_bf16_is_rounded_f32():
    K = _K()
    g = torch.Generator(device="cuda").manual_seed(2)
    rows, d = 3001, 1024
    y = torch.randn(rows, d, device="cuda", generator=g)
    mean, rstd = torch.randn(d, device="cuda", generator=g), torch.rand(d, device="cuda", generator=g) + 0.5
    gm, bt = torch.randn(d, device="cuda", generator=g), torch.randn(d, device="cuda", generator=g)
    z = torch.empty_like(y)
    z16 = torch.empty(y.shape, device="cuda", dtype=torch.bfloat16)
    K.bn_silu_fwd(y, mean, rstd, gm, bt, z)
    K.bn_silu_fwd(y, mean, rstd, gm, bt, z16)
    torch.cuda.synchronize()
    assert torch.equal(z16, z.bfloat16())


def test_glu_mask_bwd_bf16_is_rounded_f32():
    K = _K()
    g = torch.Generator(device="cuda").manual_seed(3)
    B, T, d = 4, 201, 1024
    dg = torch.randn(B * T, d, device="cuda", generator=g)
    a = torch.randn(B * T, 2 * d, device="cuda", generator=g)
    lens = torch.tensor([201, 150, 7, 199], dtype=torch.int64, device="cuda")
    da = torch.empty_like(a)
    da16 = torch.empty(a.shape, device="cuda", dtype=torch.bfloat16)
    K.glu_mask_bwd(dg, a, lens, da, B, T, d)
    K.glu_mask_bwd(dg, a, lens, da16, B, T, d)
    torch.cuda.synchronize()
    assert torch.equal(da16, da.bfloat16())
