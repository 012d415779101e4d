"""Fused Conformer macaron FFN block (csrc/ffn.hip: LayerNorm -> Linear -> SiLU -> dropout -> Linear ->
dropout -> 0.5-scaled residual, forward + data-gradient/LayerNorm backward in one launch each).

Reference: the feed_forward1 / feed_forward2 half steps of ConformerLayer.forward (NeMo
conformer_modules.py ConformerFeedForward), written out in torch float64 and
differentiated by autograd.  Tolerances (bf16 MFMA operands, f32 accumulation): output and every
gradient relative Frobenius error <= 2e-2 against float64; the weight gradients go through
kdfm_wgrad_bf16 on the bf16 operands the backward kernel writes.  With dropout on, the fused block is
compared with the unfused bf16 GPU path (LN + two kdfm_gemm launches + dropout / dSiLU epilogues),
which draws the same counter-RNG masks: the masks must agree exactly (zero pattern of the hidden
activation) and the values to bf16 accuracy.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _params(d, ff, g):
    return {
        "ln_g": 1.0 + 0.1 * torch.randn(d, generator=g),
        "ln_b": 0.1 * torch.randn(d, generator=g),
        "W1": torch.randn(ff, d, generator=g) / d ** 0.5,
        "b1": 0.1 * torch.randn(ff, generator=g),
        "W2": torch.randn(d, ff, generator=g) / ff ** 0.5,
        "b2": 0.1 * torch.randn(d, generator=g),
    }


def _ref(P, x, dout, eps=1e-5):
    P = {k: v.double().clone().requires_grad_(True) for k, v in P.items()}
    x = x.double().clone().requires_grad_(True)
    ln = torch.nn.functional.layer_norm(x, (x.shape[1],), P["ln_g"], P["ln_b"], eps)
    a = torch.nn.functional.silu(ln @ P["W1"].t() + P["b1"])
    out = x + 0.5 * (a @ P["W2"].t() + P["b2"])
    grads = torch.autograd.grad(out, [x] + list(P.values()), dout.double())
    return out.detach(), dict(zip(["x"] + list(P), grads))


def _fused(P, x, dout, *, p=0.0, seed=None):
    from kdfm import kernels as K
    rows, d = x.shape
    ff = P["W1"].shape[0]
    dev = x.device
    img = K.ffn_img(P["W1"], P["W2"])
    out = torch.empty_like(x)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    K.ffn_fwd(x, P["ln_g"], P["ln_b"], 1e-5, img, P["b1"], P["b2"], out, mean, rstd, ff, rscale=0.5, p_act=p, p_out=p,
              seed=seed, st_act=101, st_out=102)
    bf = torch.bfloat16
    ln_h = torch.empty(rows, d, device=dev, dtype=bf)
    dl2_h = torch.empty(rows, d, device=dev, dtype=bf)
    a_h = torch.empty(rows, ff, device=dev, dtype=bf)
    dh_h = torch.empty(rows, ff, device=dev, dtype=bf)
    dx = torch.empty_like(x)
    part = torch.empty(K.layernorm_bwd_ws(rows, d), device=dev)
    K.ffn_bwd(dout, x, mean, rstd, P["ln_g"], P["ln_b"], img, P["b1"], dx, ln_h, a_h, dl2_h, dh_h, part, ff, rscale=0.5,
              p_act=p, p_out=p, seed=seed, st_act=101, st_out=102)
    G = {k: torch.zeros_like(v) for k, v in P.items()}
    if K.wgrad_bf16_supported(rows, d, ff) and K.wgrad_bf16_supported(rows, ff, d):
        K.wgrad_bf16(dl2_h, a_h, G["W2"], db=G["b2"])
        K.wgrad_bf16(dh_h, ln_h, G["W1"], db=G["b1"])
    else:   # wider than the row-parallel kernel's tiles (the engine then keeps the unfused backward)
        G["W2"], G["b2"] = dl2_h.double().t() @ a_h.double(), dl2_h.double().sum(0)
        G["W1"], G["b1"] = dh_h.double().t() @ ln_h.double(), dh_h.double().sum(0)
    K.ln_fold([(part, G["ln_g"], G["ln_b"])], rows, d)
    torch.cuda.synchronize()
    return out, dx, G, dict(mean=mean, rstd=rstd, a_h=a_h, dh_h=dh_h)


@pytest.mark.parametrize("rows,d", [(12832, 88), (1000, 88), (37, 88), (4010, 176), (130, 192)])
def test_ffn_block_matches_float64(rows, d):
    from kdfm import kernels as K
    ff = 4 * d
    assert K.ffn_supported(d, ff)
    g = torch.Generator().manual_seed(rows + d)
    P = _params(d, ff, g)
    x = torch.randn(rows, d, generator=g) * 2.0 + 0.3
    dout = torch.randn(rows, d, generator=g)
    ref_out, ref_g = _ref(P, x, dout)
    Pc = {k: v.cuda() for k, v in P.items()}
    out, dx, G, aux = _fused(Pc, x.cuda(), dout.cuda())
    assert _rel(out - x.cuda(), ref_out - x.double()) <= 2e-2
    xd = x.double()
    assert _rel(aux["mean"], xd.mean(1)) <= 1e-6
    assert _rel(aux["rstd"], 1.0 / (xd.var(1, unbiased=False) + 1e-5).sqrt()) <= 1e-5
    assert _rel(dx - dout.cuda(), ref_g["x"] - dout.double()) <= 2e-2
    for k in P:
        assert _rel(G[k], ref_g[k]) <= 2e-2, k


def test_ffn_block_dropout_matches_unfused_path():
    """Same counter-RNG masks as the unfused LN + kdfm_gemm path (conformer.py with KDFM_FFN_FUSED=0)."""
    from kdfm import _lib
    from kdfm import kernels as K
    rows, d = 3001, 88
    ff = 4 * d
    g = torch.Generator().manual_seed(7)
    P = {k: v.cuda() for k, v in _params(d, ff, g).items()}
    x = (torch.randn(rows, d, generator=g) + 0.1).cuda()
    dout = torch.randn(rows, d, generator=g).cuda()
    seed = torch.tensor([123456789], dtype=torch.int64, device="cuda")
    p = 0.1
    with K.mode(math="bf16"):
        out, dx, G, aux = _fused(P, x, dout, p=p, seed=seed)
        # unfused reference on the same kernels the f32-storage path uses
        ln = torch.empty_like(x)
        m = torch.empty(rows, device="cuda")
        r = torch.empty(rows, device="cuda")
        K.layernorm_fwd(x, P["ln_g"], P["ln_b"], ln, m, r, 1e-5)
        h = torch.empty(rows, ff, device="cuda")
        a = torch.empty(rows, ff, device="cuda")
        K.linear(ln, P["W1"], P["b1"], a, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE, Cpre=h, dropout_p=p, seed=seed,
                 rng_stream=101)
        out_u = torch.empty_like(x)
        K.linear(a, P["W2"], P["b2"], out_u, epi=_lib.EPI_RESID, R=x, rscale=0.5, dropout_p=p, seed=seed,
                 rng_stream=102)
        dl2 = torch.empty_like(x)
        K.dropout(dout, dl2, p, 0.5, seed, 102)
        dh = torch.empty(rows, ff, device="cuda")
        K.linear_dx(dl2, P["W2"], dh, epi=_lib.EPI_DSILU, aux=h, dropout_p=p, seed=seed, rng_stream=101)
        torch.cuda.synchronize()
    # identical masks: the hidden activation is zero exactly where the unfused one is
    zf = aux["a_h"].float() == 0
    zu = a == 0
    assert torch.equal(zf, zu)
    assert 0.08 < zu.float().mean().item() < 0.12
    assert _rel(aux["a_h"].float(), a) <= 1e-2
    assert torch.equal(aux["dh_h"].float() == 0, dh == 0)
    assert _rel(aux["dh_h"].float(), dh) <= 2e-2
    assert _rel(out - x, out_u - x) <= 1e-2
    assert _rel(aux["mean"], m) <= 1e-6 and _rel(aux["rstd"], r) <= 1e-6


def test_ffn_forward_only_image_and_no_stats():
    """Teacher mode: forward-only image (half of every chunk written), no mean / rstd saved."""
    from kdfm import kernels as K
    rows, d = 2049, 176
    ff = 4 * d
    g = torch.Generator().manual_seed(3)
    P = _params(d, ff, g)
    x = torch.randn(rows, d, generator=g)
    ref_out, _ = _ref(P, x, torch.zeros(rows, d))
    Pc = {k: v.cuda() for k, v in P.items()}
    img = K.ffn_img(Pc["W1"], Pc["W2"], fwd_only=True)
    out = torch.empty(rows, d, device="cuda")
    K.ffn_fwd(x.cuda(), Pc["ln_g"], Pc["ln_b"], 1e-5, img, Pc["b1"], Pc["b2"], out, None, None, ff, rscale=0.5,
              p_act=0.0, p_out=0.0, seed=None, st_act=0, st_out=0)
    torch.cuda.synchronize()
    assert _rel(out - x.cuda(), ref_out - x.double()) <= 2e-2


def test_ffn_unsupported_shape_raises():
    from kdfm import _lib
    from kdfm import kernels as K
    assert not K.ffn_supported(64, 256)
    W1 = torch.zeros(256, 64, device="cuda")
    W2 = torch.zeros(64, 256, device="cuda")
    with pytest.raises(_lib.KdfmError):
        K.ffn_img(W1, W2)


@pytest.mark.parametrize("rows,d", [(12832, 88), (37, 88), (2049, 176)])
def test_ffn_block_fused_norm_out(rows, d):
    """The layer's norm_out LayerNorm computed in the FFN2 epilogue (kdfm_ffn_fwd out_ln): the block
    output, LN(output) and its row statistics against float64."""
    from kdfm import kernels as K
    ff = 4 * d
    g = torch.Generator().manual_seed(5 * rows + d)
    P = _params(d, ff, g)
    x = torch.randn(rows, d, generator=g)
    g5 = 1.0 + 0.1 * torch.randn(d, generator=g)
    b5 = 0.1 * torch.randn(d, generator=g)
    ref_out, _ = _ref(P, x, torch.zeros(rows, d))
    ref_y = torch.nn.functional.layer_norm(ref_out, (d,), g5.double(), b5.double(), 1e-5)
    Pc = {k: v.cuda() for k, v in P.items()}
    out = torch.empty(rows, d, device="cuda")
    y = torch.empty(rows, d, device="cuda")
    m5, r5 = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    K.ffn_fwd(x.cuda(), Pc["ln_g"], Pc["ln_b"], 1e-5, K.ffn_img(Pc["W1"], Pc["W2"], fwd_only=True), Pc["b1"], Pc["b2"],
              out, None, None, ff, rscale=0.5, p_act=0.0, p_out=0.0, seed=None, st_act=0, st_out=0,
              out_ln=(g5.cuda(), b5.cuda(), 1e-5, y, m5, r5))
    torch.cuda.synchronize()
    assert _rel(out - x.cuda(), ref_out - x.double()) <= 2e-2
    # LN of the kernel's own output in float64 (the statistics must match what it normalised)
    own = torch.nn.functional.layer_norm(out.double().cpu(), (d,), g5.double(), b5.double(), 1e-5)
    assert _rel(y, own) <= 1e-6
    assert _rel(y, ref_y) <= 2e-2
    assert _rel(m5, out.double().mean(1)) <= 1e-6
    assert _rel(r5, 1.0 / (out.double().var(1, unbiased=False) + 1e-5).sqrt()) <= 1e-5
