"""Thin, typed Python wrappers over the libkdfm.so C-ABI (no autograd here).

Tensors are torch CUDA tensors used purely as device allocations; every arithmetic operation
runs in a libkdfm kernel on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import GemmDesc, call

_MATH = {"f32": _lib.KDFM_MATH_F32, "bf16": _lib.KDFM_MATH_BF16}


class _State:
    math = "f32"


def set_math(mode: str) -> None:
    if mode not in _MATH:
        raise ValueError(f"math mode must be one of {list(_MATH)}")
    _State.math = mode


def get_math() -> str:
    return _State.math


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.KdfmError("kdfm kernels need device tensors (HIP); got a CPU tensor")
    if t.dtype not in (torch.float32, torch.int64, torch.int32, torch.uint64, torch.uint8, torch.bool):
        raise _lib.KdfmError(f"unsupported dtype {t.dtype}")
    return t.data_ptr()


def gemm(A, B, Cout, M, N, K, sAm, sAk, sBk, sBn, sCm, sCn, *, amode, bmode,
         batch=(1, 1), bA=(0, 0), bB=(0, 0), bC=(0, 0), alpha=1.0, epi=0, bias=None, R=None, rscale=1.0,
         aux=None, Cpre=None, beta=0.0, dropout_p=0.0, seed=None, rng_stream=0, splitk=1,
         conv=None, math=None):
    d = GemmDesc()
    d.A, d.B, d.C = ptr(A), ptr(B), ptr(Cout)
    d.bias, d.R, d.aux, d.Cpre = ptr(bias), ptr(R), ptr(aux), ptr(Cpre)
    d.M, d.N, d.K = M, N, K
    d.sAm, d.sAk, d.sBk, d.sBn, d.sCm, d.sCn = sAm, sAk, sBk, sBn, sCm, sCn
    d.batch1, d.batch2 = batch
    d.bA1, d.bA2 = bA
    d.bB1, d.bB2 = bB
    d.bC1, d.bC2 = bC
    d.alpha, d.beta, d.rscale, d.dropout_p = alpha, beta, rscale, dropout_p
    d.seed = ptr(seed)
    d.rng_stream = rng_stream
    d.amode, d.bmode, d.epi = amode, bmode, epi
    d.math = _MATH[math or _State.math]
    d.splitk = splitk
    if conv is not None:
        d.conv_taps, d.conv_pad, d.conv_c, d.conv_t = conv
    call("kdfm_gemm", C.byref(d), stream_ptr())


def _splitk_for(M, N, K):
    tiles = -(-M // 64) * -(-N // 64)
    if K <= 256 or tiles >= 512:
        return 1
    want = max(1, 1024 // tiles)
    return int(min(want, max(1, K // 256), 256))


# ---------------- Linear-layer products on row-major 2-D views ---------------------------------

def linear_fwd(x, W, bias, out, *, epi=0, R=None, rscale=1.0, Cpre=None, dropout_p=0.0, seed=None,
               rng_stream=0, math=None):
    """out[M,N] = epi(x[M,K] @ W[N,K]^T + bias)"""
    M, K = x.shape
    N = W.shape[0]
    if bias is not None:
        epi |= _lib.EPI_BIAS
    gemm(x, W, out, M, N, K, x.stride(0), x.stride(1), W.stride(1), W.stride(0), out.stride(0), out.stride(1),
         amode=_lib.LD_KC, bmode=_lib.LD_KC, epi=epi, bias=bias, R=R, rscale=rscale, Cpre=Cpre,
         dropout_p=dropout_p, seed=seed, rng_stream=rng_stream, math=math)


def linear_dx(dy, W, dx, *, epi=0, aux=None, dropout_p=0.0, seed=None, rng_stream=0, beta=0.0, R=None,
              rscale=1.0, math=None):
    """dx[M,K] = epi(dy[M,N] @ W[N,K])"""
    M, N = dy.shape
    K = W.shape[1]
    gemm(dy, W, dx, M, K, N, dy.stride(0), dy.stride(1), W.stride(0), W.stride(1), dx.stride(0), dx.stride(1),
         amode=_lib.LD_KC, bmode=_lib.LD_XC, epi=epi, aux=aux, dropout_p=dropout_p, seed=seed,
         rng_stream=rng_stream, beta=beta, R=R, rscale=rscale, math=math)


def linear_dw(dy, x, dW, *, accumulate=False, math=None):
    """dW[N,K] (+)= dy[M,N]^T @ x[M,K]   (split-K with f32 atomics)"""
    M, N = dy.shape
    K = x.shape[1]
    if not accumulate:
        dW.zero_()  # noqa: kernel-side memset via torch allocator (hipMemsetAsync)
    sk = _splitk_for(N, K, M)
    gemm(dy, x, dW, N, K, M, dy.stride(1), dy.stride(0), x.stride(0), x.stride(1), dW.stride(0), dW.stride(1),
         amode=_lib.LD_XC, bmode=_lib.LD_XC, epi=_lib.EPI_ATOMIC, splitk=sk, math=math)


def colsum(x2d, out, accumulate=False):
    M, N = x2d.shape
    assert x2d.stride(1) == 1
    call("kdfm_colsum", ptr(x2d), ptr(out), M, N, x2d.stride(0), int(accumulate), stream_ptr())
