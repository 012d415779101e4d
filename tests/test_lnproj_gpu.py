"""LayerNorm-fused input projections (csrc/lnproj.hip) against float64 torch references.

QKV: ln = LN(x); q|k|v = ln W^T + b; qu = q + pos_bias_u, qv = q + pos_bias_v (RelPositionMultiHeadAttention
linear_q/k/v and the positional biases).  GLU: ln = LN(x); a|gate = ln W^T + b;
g = a sigmoid(gate) zeroed on padded frames (ConformerConvolution pointwise_conv1 + GLU + pad mask,
Appendix A.6).  Backward: dx = dres + LN'(W^T dproj) and the parameter gradients (weights through
kdfm_wgrad_bf16 on the bf16 operands the kernel writes, LN dgamma/dbeta through kdfm_ln_fold).
Tolerance: relative Frobenius error <= 2e-2 (bf16 MFMA operands, f32 accumulation).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _setup(kind, B, T, d, seed):
    g = torch.Generator().manual_seed(seed)
    n = (3 if kind == 0 else 2) * d
    P = {"ln_g": 1.0 + 0.1 * torch.randn(d, generator=g), "ln_b": 0.1 * torch.randn(d, generator=g),
         "W": torch.randn(n, d, generator=g) / d ** 0.5, "b": 0.1 * torch.randn(n, generator=g)}
    if kind == 0:
        P["u"] = 0.1 * torch.randn(d, generator=g)
        P["v"] = 0.1 * torch.randn(d, generator=g)
    x = 1.5 * torch.randn(B * T, d, generator=g) + 0.2
    lens = torch.randint(T // 2, T + 1, (B,), generator=g)
    lens[0] = T
    return P, x, lens


def _ref_fwd(kind, P, x, lens, T):
    d = x.shape[1]
    P = {k: v.double().clone().requires_grad_(True) for k, v in P.items()}
    x = x.double().clone().requires_grad_(True)
    ln = torch.nn.functional.layer_norm(x, (d,), P["ln_g"], P["ln_b"], 1e-5)
    y = ln @ P["W"].t() + P["b"]
    if kind == 0:
        q = y[:, :d]
        outs = {"qu": q + P["u"], "qv": q + P["v"], "k": y[:, d:2 * d], "vv": y[:, 2 * d:]}
    else:
        live = (torch.arange(x.shape[0]) % T < lens.repeat_interleave(T)).double()[:, None]
        outs = {"g": y[:, :d] * torch.sigmoid(y[:, d:]) * live}
    return outs, P, x


@pytest.mark.parametrize("B,T,d", [(32, 401, 88), (3, 37, 88), (4, 101, 176)])
def test_ln_qkv_forward(B, T, d):
    from kdfm import kernels as K
    P, x, lens = _setup(0, B, T, d, B + T + d)
    ref, _, _ = _ref_fwd(0, P, x, lens, T)
    Pc = {k: v.cuda() for k, v in P.items()}
    rows = B * T
    qu, qv = torch.empty(rows, d, device="cuda"), torch.empty(rows, d, device="cuda")
    qkv = torch.zeros(rows, 3 * d, device="cuda")
    mean, rstd = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    lnh = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    K.ln_qkv_fwd(x.cuda(), Pc["ln_g"], Pc["ln_b"], 1e-5, K.lnproj_img(0, Pc["W"]), Pc["b"], Pc["u"], Pc["v"], qu, qv,
                 qkv, mean, rstd, lnh)
    torch.cuda.synchronize()
    assert _rel(qu, ref["qu"]) <= 2e-2 and _rel(qv, ref["qv"]) <= 2e-2
    assert _rel(qkv[:, d:2 * d], ref["k"]) <= 2e-2 and _rel(qkv[:, 2 * d:], ref["vv"]) <= 2e-2
    assert _rel(mean, x.double().mean(1)) <= 1e-6
    ln = torch.nn.functional.layer_norm(x.double(), (d,), P["ln_g"].double(), P["ln_b"].double(), 1e-5)
    assert _rel(lnh.float(), ln) <= 5e-3


@pytest.mark.parametrize("B,T,d", [(32, 401, 88), (3, 37, 88), (4, 101, 176)])
def test_ln_glu_forward(B, T, d):
    from kdfm import kernels as K
    P, x, lens = _setup(1, B, T, d, 7 * B + T + d)
    ref, _, _ = _ref_fwd(1, P, x, lens, T)
    Pc = {k: v.cuda() for k, v in P.items()}
    rows = B * T
    gout = torch.empty(rows, d, device="cuda")
    K.ln_glu_fwd(x.cuda(), Pc["ln_g"], Pc["ln_b"], 1e-5, K.lnproj_img(1, Pc["W"]), Pc["b"], lens.cuda(), T, gout)
    torch.cuda.synchronize()
    assert _rel(gout, ref["g"]) <= 2e-2
    live = torch.arange(rows) % T < lens.repeat_interleave(T)
    assert torch.all(gout.cpu()[~live] == 0)


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("B,T", [(32, 401), (3, 37)])
def test_lnproj_backward(kind, B, T):
    from kdfm import kernels as K
    d = 88
    rows = B * T
    P, x, lens = _setup(kind, B, T, d, 11 * B + T + kind)
    outs, Pd, xd = _ref_fwd(kind, P, x, lens, T)
    g = torch.Generator().manual_seed(5)
    grads_out = {k: torch.randn(v.shape, generator=g, dtype=torch.float64) for k, v in outs.items()}
    dres = torch.randn(rows, d, generator=g)
    total = sum((outs[k] * grads_out[k]).sum() for k in outs)
    names = list(Pd)
    ref = dict(zip(["x"] + names, torch.autograd.grad(total, [xd] + [Pd[k] for k in names])))
    Pc = {k: v.cuda() for k, v in P.items()}
    xc = x.cuda()
    mean, rstd = torch.empty(rows, device="cuda"), torch.empty(rows, device="cuda")
    lens_c = lens.cuda()
    # forward only for the row statistics
    if kind == 0:
        qu, qv = torch.empty(rows, d, device="cuda"), torch.empty(rows, d, device="cuda")
        qkv = torch.empty(rows, 3 * d, device="cuda")
        K.ln_qkv_fwd(xc, Pc["ln_g"], Pc["ln_b"], 1e-5, K.lnproj_img(0, Pc["W"]), Pc["b"], Pc["u"], Pc["v"], qu, qv, qkv,
                     mean, rstd)
    else:
        gout = torch.empty(rows, d, device="cuda")
        K.ln_glu_fwd(xc, Pc["ln_g"], Pc["ln_b"], 1e-5, K.lnproj_img(1, Pc["W"]), Pc["b"], lens_c, T, gout, mean, rstd)
    n = (3 if kind == 0 else 2) * d
    dx = torch.empty(rows, d, device="cuda")
    lnh = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
    dph = torch.empty(rows, n, device="cuda", dtype=torch.bfloat16)
    part = torch.empty(K.layernorm_bwd_ws(rows, d), device="cuda")
    img = K.lnproj_img(kind, Pc["W"], bwd=True)
    if kind == 0:
        dqkv = torch.zeros(rows, 3 * d)
        dqkv[:, d:2 * d] = grads_out["k"].float()
        dqkv[:, 2 * d:] = grads_out["vv"].float()
        part_uv = torch.empty(K.layernorm_bwd_ws(rows, d), device="cuda")
        K.ln_qkv_bwd(grads_out["qu"].float().cuda(), grads_out["qv"].float().cuda(), dqkv.cuda(), xc, mean, rstd,
                     Pc["ln_g"], Pc["ln_b"], img, dres.cuda(), dx, lnh, dph, part, part_uv)
    else:
        K.ln_glu_bwd(grads_out["g"].float().cuda(), xc, mean, rstd, Pc["ln_g"], Pc["ln_b"], img, Pc["b"], lens_c, T,
                     dres.cuda(), dx, lnh, dph, part)
    GW = torch.zeros(n, d, device="cuda")
    Gb = torch.zeros(n, device="cuda")
    K.wgrad_bf16(dph, lnh, GW, db=Gb)
    Gg = torch.zeros(d, device="cuda")
    Gbeta = torch.zeros(d, device="cuda")
    entries = [(part, Gg, Gbeta)]
    if kind == 0:   # positional-bias gradients folded with the LN partials
        Gu = torch.full((d,), 0.25, device="cuda")
        Gv = torch.zeros(d, device="cuda")
        entries.append((part_uv, Gu, Gv))
    K.ln_fold(entries, rows, d)
    torch.cuda.synchronize()
    if kind == 0:
        assert _rel(Gu - 0.25, ref["u"]) <= 1e-5 and _rel(Gv, ref["v"]) <= 1e-5
    assert _rel(dx - dres.cuda(), ref["x"]) <= 2e-2
    assert _rel(GW, ref["W"]) <= 2e-2
    assert _rel(Gb, ref["b"]) <= 2e-2
    assert _rel(Gg, ref["ln_g"]) <= 2e-2
    assert _rel(Gbeta, ref["ln_b"]) <= 2e-2


def test_batched_weight_images_match_single_preps():
    """kdfm_wimg_prep_batch (one launch for every image of an encoder) writes the same bytes as the
    per-image prep entry points, for the student (training images) and the teacher (forward-only)."""
    from kdfm import kernels as K
    from kdfm.config import DEFAULT
    from kdfm.conformer import layer_images
    from kdfm.store import FlatStore
    from kdfm.config import student_specs, teacher_specs
    from dataclasses import replace
    cfg = replace(DEFAULT, n_layers=2)
    for specs, prefix, d, train in ((student_specs(cfg), "encoder.", cfg.d_student, True),
                                    (teacher_specs(cfg), "teacher.encoder.", cfg.d_teacher, False)):
        st = FlatStore(specs, "cuda", with_grad=False)
        st.data.copy_(torch.randn(st.numel, generator=torch.Generator().manual_seed(d)))
        imgs = layer_images(cfg, st.P, prefix, d, train=train, dev=torch.device("cuda"))
        imgs.refresh()
        torch.cuda.synchronize()
        saved, K._IMGSETS[:] = list(K._IMGSETS), []   # per-image preps, not the registered batch
        try:
            for key, typ, kind, flag, dd, ff, W1, W2 in imgs.specs:
                if typ == K.IMG_FFN:
                    ref = K.ffn_img(W1, W2, fwd_only=bool(flag))
                    if flag:   # forward-only: compare the forward halves of every chunk
                        KS1, DT = (6, 3) if d <= 96 else (11, 6)
                        cs, fw = 4 * DT + 2 * KS1, 2 * DT + KS1
                        a = imgs.get(key).view(-1, cs, 512)[:, :fw]
                        b = ref.view(-1, cs, 512)[:, :fw]
                        assert torch.equal(a, b), key
                        continue
                elif typ == K.IMG_LNPROJ:
                    ref = K.lnproj_img(kind, W1, bwd=bool(flag))
                else:
                    ref = K.rowgemm_img(W1, trans=bool(flag))
                torch.cuda.synchronize()
                assert torch.equal(imgs.get(key), ref), key
        finally:
            K._IMGSETS[:] = saved
