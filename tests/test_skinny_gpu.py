"""GPU numerics of the weight-stationary skinny GEMM (csrc/skinny.hip) that kdfm_gemm selects for
bf16 products with M >= 2048 rows: every encoder Linear / 1x1 conv (M = B*T' = 12,832 at the bench
config), the KD heads (M = 16*B*T') and their data-gradients.  Reference: torch fp32 matmul of
the SAME bf16-rounded operands (only the f32 accumulation order differs: tolerance 2e-3 of
max |ref|).  Dropout masks are checked against the exact-f32 generic kernel (same counter RNG)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from kdfm import kernels
    return kernels


def _bf(t):
    return t.to(torch.bfloat16).float()


def _close(out, ref, rel=2e-3):
    tol = rel * ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


# (M, N, K): student / teacher encoder products (d = 88 / 176, FFN 4d, qkv 3d, pw1 2d), decoder,
# ragged M, and K spanning several 96-wide chunks.
SHAPES = [(12832, 88, 88), (12832, 352, 88), (12832, 88, 352), (12832, 264, 88), (12832, 176, 88),
          (12832, 176, 176), (12832, 704, 176), (12832, 176, 704), (12832, 528, 176), (12832, 129, 88),
          (2053, 40, 24), (4099, 96, 200)]


@pytest.mark.parametrize("M,N,Kd", SHAPES)
def test_skinny_linear(K, M, N, Kd):
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + Kd)
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    y = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, y, epi=_lib.EPI_SILU, math="bf16")
    h = _bf(x) @ _bf(W).T + b
    _close(y, torch.nn.functional.silu(h))
    # residual epilogue (out = R + rscale * (xW^T + b))
    R = torch.randn(M, N, device="cuda", generator=g)
    K.linear(x, W, b, y, R=R, rscale=0.5, epi=_lib.EPI_RESID, math="bf16")
    _close(y, R + 0.5 * h)


@pytest.mark.parametrize("M,N,Kd", SHAPES[:9])
def test_skinny_linear_dx(K, M, N, Kd):
    """dx = dy @ W with B contiguous along n (XC), dSiLU epilogue"""
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(7 * M + N + Kd)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    dy = torch.randn(M, N, device="cuda", generator=g)
    aux = torch.randn(M, Kd, device="cuda", generator=g)
    dx = torch.empty(M, Kd, device="cuda")
    K.linear_dx(dy, W, dx, epi=_lib.EPI_DSILU, aux=aux, math="bf16")
    s = torch.sigmoid(aux)
    _close(dx, (_bf(dy) @ _bf(W)) * s * (1 + aux * (1 - s)))


def test_skinny_strided_views(K):
    """A as a column slice of a wider row-major buffer (qkv[:, d:]-style views) and C strided."""
    g = torch.Generator(device="cuda").manual_seed(11)
    M, d = 12832, 88
    big = torch.randn(M, 3 * d, device="cuda", generator=g)
    x = big[:, d:2 * d]
    W = torch.randn(d, d, device="cuda", generator=g) * 0.1
    outbig = torch.zeros(M, 2 * d, device="cuda")
    y = outbig[:, d:]
    K.linear(x, W, None, y, math="bf16")
    _close(y, _bf(x) @ _bf(W).T)
    assert outbig[:, :d].abs().max().item() == 0.0


def test_skinny_dropout_matches_generic(K):
    """The counter-RNG dropout mask depends only on (seed, stream, row, col): the skinny bf16 path
    and the generic exact-f32 path must drop exactly the same elements."""
    from kdfm import _lib
    g = torch.Generator(device="cuda").manual_seed(3)
    M, N, Kd = 12832, 352, 88
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g) + 3.0     # keep SiLU outputs away from 0
    seed = torch.tensor([12345], dtype=torch.int64, device="cuda")
    pre_bf = torch.empty(M, N, device="cuda")
    y_bf = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, y_bf, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE, Cpre=pre_bf, dropout_p=0.1, seed=seed,
             rng_stream=77, math="bf16")
    pre_f = torch.empty(M, N, device="cuda")
    y_f = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, y_f, epi=_lib.EPI_SILU | _lib.EPI_STORE_PRE, Cpre=pre_f, dropout_p=0.1, seed=seed,
             rng_stream=77, math="f32")
    assert torch.equal(y_bf == 0, y_f == 0)
    frac = (y_bf == 0).float().mean().item()
    assert 0.08 < frac < 0.12
    _close(pre_bf, _bf(x) @ _bf(W).T + b)
    _close(y_bf, y_f, rel=1e-2)


def test_skinny_rowmask_and_mse(K):
    g = torch.Generator(device="cuda").manual_seed(4)
    U, T, N, Kd = 32, 401, 96, 96
    M = U * T
    x = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    lens = torch.randint(100, T + 1, (U,), generator=torch.Generator().manual_seed(0)).to("cuda")
    y = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, y, rowmask=(lens, T, 1), math="bf16")
    ref = (_bf(x) @ _bf(W).T + b).view(U, T, N)
    keep = (torch.arange(T, device="cuda")[None, :] < lens[:, None]).float()[..., None]
    _close(y, (ref * keep).view(M, N))
    tgt = torch.randn(M, N, device="cuda", generator=g)
    acc = torch.zeros(1, device="cuda")
    d = torch.empty(M, N, device="cuda")
    K.linear(x, W, b, d, R=tgt, rscale=2.0 / (M * N), mse=(acc, 1.0 / (M * N)), math="bf16")
    diff = _bf(x) @ _bf(W).T + b - tgt
    _close(d, diff * 2.0 / (M * N))
    assert abs(acc.item() - (diff ** 2).mean().item()) <= 1e-4 * (diff ** 2).mean().item()


def _twin_buffer(shapes, seed):
    """A flat f32 buffer holding weights of the given 2-D shapes, with registered bf16 twins
    (same layout + per-weight transposes), like FlatStore.enable_bf16_twins."""
    from kdfm import kernels as Kk
    g = torch.Generator(device="cuda").manual_seed(seed)
    offs, off = [], 0
    for r, c in shapes:
        offs.append(off)
        off += -(-(r * c) // 4) * 4
    src = torch.randn(off, device="cuda", generator=g) * 0.1
    h = torch.empty(off, device="cuda", dtype=torch.bfloat16)
    ht = torch.empty(off, device="cuda", dtype=torch.bfloat16)
    entries = [(o, r, c) for o, (r, c) in zip(offs, shapes)]
    tab, blk = [], 0
    for o, r, c in entries:
        tab.append((o, r, c, blk))
        blk += -(-(r * c) // 256)
    Kk.register_bf16_twin(src, h, ht, entries)
    Kk.cast_bf16(src, h)
    Kk.cast_bf16_t(src, ht, torch.tensor(tab, dtype=torch.int64, device="cuda"), len(tab), blk)
    Ws = [src[o:o + r * c].view(r, c) for o, (r, c) in zip(offs, shapes)]
    return src, h, ht, Ws


@pytest.mark.parametrize("M", [12832, 205312 // 4, 3001])
def test_skinny_direct_twins(K, M):
    """Forward (B = W rows) and data-gradient (B = W^T rows) products reading the bf16 twins, incl.
    a column-slice view (W1[:, :96] of a (96, 128) weight, the FM meta-encoder's x part)."""
    from kdfm import _lib
    d = 88
    shapes = [(4 * d, d), (d, 4 * d), (3 * d, d), (129, d), (96, 128), (96, 176)]
    src, h, ht, Ws = _twin_buffer(shapes, M)
    assert torch.equal(h.float(), _bf(src))
    g = torch.Generator(device="cuda").manual_seed(1)
    for W in Ws[:4] + [Ws[4][:, :96], Ws[5]]:
        N, Kd = W.shape
        x = torch.randn(M, Kd, device="cuda", generator=g)
        b = torch.randn(N, device="cuda", generator=g)
        R = torch.randn(M, N, device="cuda", generator=g)
        y = torch.empty(M, N, device="cuda")
        K.linear(x, W, b, y, R=R, rscale=-0.25, epi=_lib.EPI_RESID, math="bf16")
        _close(y, R - 0.25 * (_bf(x) @ _bf(W).T + b))
        dy = torch.randn(M, N, device="cuda", generator=g)
        aux = torch.randn(M, Kd, device="cuda", generator=g)
        dx = torch.empty(M, Kd, device="cuda")
        K.linear_dx(dy, W, dx, epi=_lib.EPI_DRELU, aux=aux, alpha=0.5, math="bf16")
        _close(dx, torch.where(aux > 0, 0.5 * (_bf(dy) @ _bf(W)), torch.zeros_like(aux)))
    del src


def test_skinny_direct_conv3_twin(K):
    from kdfm import kernels as Kk
    T, U, C = 401, 40, 96
    M = T * U
    g = torch.Generator(device="cuda").manual_seed(9)
    wconv = torch.randn(2, C, 3 * C, device="cuda", generator=g) * 0.05
    wh = torch.empty(2, C, 3 * C, device="cuda", dtype=torch.bfloat16)
    Kk.register_bf16_twin(wconv, wh)
    Kk.cast_bf16(wconv, wh)
    x = torch.randn(M, C, device="cuda", generator=g)
    b = torch.randn(C, device="cuda", generator=g)
    out = torch.empty(M, C, device="cuda")
    from kdfm import _lib
    K.conv3(x, wconv[1], b, out, T, epi=_lib.EPI_RELU, math="bf16")
    xs = torch.nn.functional.pad(_bf(x).view(U, T, C), (0, 0, 1, 1))
    taps = torch.cat([xs[:, t:t + T] for t in range(3)], dim=2).reshape(M, 3 * C)
    _close(out, torch.relu(taps @ _bf(wconv[1]).T + b))


@pytest.mark.parametrize("T,U", [(401, 164), (7, 9363), (33, 2000)])
def test_skinny_conv3_slab(K, T, U):
    """LDS-slab CONV kernel (skc_fwd_kernel: M >= 65536 rows, N <= 96, the denoiser convs of
    asr_train_diffm.py:444-460 stacked over layers): each epilogue the heads use, utterance
    boundaries inside a 32-row tile (T = 7, 33) and a ragged last tile (M % 32 != 0)."""
    from kdfm import _lib
    C = 96
    M = T * U
    g = torch.Generator(device="cuda").manual_seed(11)
    Wf = torch.randn(C, 3 * C, device="cuda", generator=g) * 0.05
    x = torch.randn(M, C, device="cuda", generator=g)
    b = torch.randn(C, device="cuda", generator=g)
    R = torch.randn(M, C, device="cuda", generator=g)
    xs = torch.nn.functional.pad(_bf(x).view(U, T, C), (0, 0, 1, 1))
    taps = torch.cat([xs[:, t:t + T] for t in range(3)], dim=2).reshape(M, 3 * C)
    ref = taps @ _bf(Wf).T
    del xs, taps
    out = torch.empty(M, C, device="cuda")
    K.conv3(x, Wf, b, out, T, epi=_lib.EPI_RELU, math="bf16")
    _close(out, torch.relu(ref + b))
    K.conv3(x, Wf, b, out, T, R=R, rscale=-1.0 / 9, math="bf16")
    _close(out, R - (ref + b) / 9)
    K.conv3(x, Wf, None, out, T, epi=_lib.EPI_DRELU, aux=R, alpha=-1.0 / 9, math="bf16")
    _close(out, torch.where(R > 0, -ref / 9, torch.zeros_like(R)))
    # N < 96 (one and two 32-column tiles) through the same kernel
    for n_out in (32, 70):
        o2 = torch.empty(M, n_out, device="cuda")
        K.conv3(x, Wf[:n_out].contiguous(), b[:n_out].contiguous(), o2, T, math="bf16")
        _close(o2, ref[:, :n_out] + b[:n_out])
