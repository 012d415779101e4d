// Shared pieces of the GEMM family (gemm.hip: generic 64x64-tile kernel; rowstream.hip: full-N
// row-streaming forward kernel and wide-tile weight-gradient kernel): the launch parameter block
// and the fused epilogue, so every kernel applies exactly the same per-element semantics
// (include/kdfm.h, KDFM_EPI_*).
#pragma once
#include "common.h"

namespace kdfm {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct GemmP {
  const float* A; const float* B; float* C; const float* bias; const float* R; const float* aux;
  float* Cpre;
  int64_t M, N, K;
  int64_t sAm, sAk, sBk, sBn, sCm, sCn;
  int64_t batch2;
  int64_t bA1, bA2, bB1, bB2, bC1, bC2;
  float alpha, beta, rscale, dropout_p;
  const uint64_t* seed; uint64_t rng_stream;
  int epi, splitk, taps, pad;
  int64_t conv_c, conv_t;
  const int64_t* mask_len; int64_t mask_T, mask_div;
  float* loss_acc; float loss_scale;
  float* ones_out; int64_t ones_col;
  float* ws; int64_t ws_len;
  const uint16_t* Bh; int64_t sBh;
  int partial;  // deterministic split-K: ATOMIC tiles store raw partials to ws[split][m][n] (folded in order)
  int nseg; int64_t seg_rows;  // row-parallel wgrad: per-segment bias columns ones_col .. one_col + nseg - 1
  const int64_t* k_dev;        // row-parallel wgrad: device-side row count (<= K) read at run time (NULL: K)
  int xslots;                  // row-parallel wgrad: 0 = one raw partial per split; 8 = per-XCD slots (atomics)
  // row-parallel wgrad, paired launch: a second product of the same shape (dY2, X2 -> C2 / ones_out2,
  // partials in ws2) in the same grid (blocks [S, 2S) and the fold's blockIdx.y == 1); A2 == NULL: none
  const float* A2; const float* B2; float* C2; float* ones_out2; float* ws2;
  // row-parallel wgrad, 3x3 stride-2 conv gather (kdfm_wgrad_bf16_s2conv): B column n = tap * conv_c + c of row
  // (b, t2, f2) reads X[b][2 t2 - 1 + tap / 3][2 f2 - 1 + tap % 3][c] of a (B, c2_T1, c2_F1, conv_c) image, zero
  // outside it and at frames >= c2_len[b] (c2_len NULL: no length mask)
  int64_t c2_T1, c2_F1, c2_T2, c2_F2; const int64_t* c2_len;
  int64_t c2_ld;   // the image's row stride (elements, >= conv_c)
};

// Non-atomic epilogue for one output element.  v = alpha * acc (already scaled).  bz = batch
// index (dropout RNG stream position).  Accumulates the MSE partial into mse_part.
__device__ __forceinline__ void epilogue_store(const GemmP& p, int64_t bz, int64_t m, int64_t n, int64_t off,
                                               float v, uint64_t seed, float keep_scale, float& mse_part) {
  const int epi = p.epi;
  if (epi & KDFM_EPI_BIAS) v += p.bias[n];
  if (epi & KDFM_EPI_MSE) {
    const float diff = v - p.R[off];
    mse_part += diff * diff;
    p.C[off] = p.rscale * diff;
    return;
  }
  if (epi & KDFM_EPI_STORE_PRE) p.Cpre[off] = v;
  if (epi & KDFM_EPI_RELU) v = fmaxf(v, 0.f);
  if (epi & KDFM_EPI_SILU) v = siluf_(v);
  if (epi & KDFM_EPI_DROPOUT) {
    const uint64_t idx = ((uint64_t)bz * (uint64_t)p.M + (uint64_t)m) * (uint64_t)p.N + (uint64_t)n;
    v = dropout_keep(seed, p.rng_stream, idx, p.dropout_p) ? v * keep_scale : 0.f;
  }
  if (epi & KDFM_EPI_DRELU) v = (p.aux[off] > 0.f) ? v : 0.f;
  if (epi & KDFM_EPI_DSILU) v *= dsiluf_(p.aux[off]);
  if (epi & KDFM_EPI_RESID) v = p.R[off] + p.rscale * v;
  if (epi & KDFM_EPI_BETA) v += p.beta * p.C[off];
  if (epi & KDFM_EPI_ROWMASK) {
    const int64_t fr = m / p.mask_div;
    const int64_t t = fr % p.mask_T, u = fr / p.mask_T;
    if (t >= p.mask_len[u]) v = 0.f;
  }
  p.C[off] = v;
}

// Two-phase epilogue (load every side operand of a tile, THEN compute and store).  On CDNA the
// vector-memory counter covers loads and stores alike, so a per-element load issued after earlier
// stores waits for all of them: an interleaved load/store epilogue serialises on store latency.
// The side operand an epilogue reads per element is at most one of R (RESID/MSE), aux
// (DRELU/DSILU) or C_old (BETA); epi_side_src() returns it and clears `single` when a descriptor
// needs more than one (callers then use epilogue_store).
__host__ __device__ inline const float* epi_side_src(const GemmP& p, bool& single) {
  const int e = p.epi;
  int cnt = 0;
  const float* s = nullptr;
  if (e & (KDFM_EPI_RESID | KDFM_EPI_MSE)) { ++cnt; s = p.R; }
  if (e & (KDFM_EPI_DRELU | KDFM_EPI_DSILU)) { ++cnt; s = p.aux; }
  if (e & KDFM_EPI_BETA) { ++cnt; s = p.C; }
  single = cnt <= 1;
  return s;
}

__device__ __forceinline__ bool epi_row_ok(const GemmP& p, int64_t m) {
  if (!(p.epi & KDFM_EPI_ROWMASK)) return true;
  const int64_t fr = m / p.mask_div;
  const int64_t t = fr % p.mask_T, u = fr / p.mask_T;
  return t < p.mask_len[u];
}

// Same per-element semantics as epilogue_store with the side value `sv` and bias `bn` already in
// registers.  Returns the value for C; *pre receives the pre-activation (STORE_PRE).
__device__ __forceinline__ float epi_apply(const GemmP& p, int64_t bz, int64_t m, int64_t n, float v, float bn, float sv,
                                           bool rowok, uint64_t seed, float keep_scale, float& mse_part,
                                           float& pre) {
  const int epi = p.epi;
  if (epi & KDFM_EPI_BIAS) v += bn;
  if (epi & KDFM_EPI_MSE) {
    const float diff = v - sv;
    mse_part += diff * diff;
    return p.rscale * diff;
  }
  pre = v;
  if (epi & KDFM_EPI_RELU) v = fmaxf(v, 0.f);
  if (epi & KDFM_EPI_SILU) v = siluf_(v);
  if (epi & KDFM_EPI_DROPOUT) {
    const uint64_t idx = ((uint64_t)bz * (uint64_t)p.M + (uint64_t)m) * (uint64_t)p.N + (uint64_t)n;
    v = dropout_keep(seed, p.rng_stream, idx, p.dropout_p) ? v * keep_scale : 0.f;
  }
  if (epi & KDFM_EPI_DRELU) v = (sv > 0.f) ? v : 0.f;
  if (epi & KDFM_EPI_DSILU) v *= dsiluf_(sv);
  if (epi & KDFM_EPI_RESID) v = sv + p.rscale * v;
  if (epi & KDFM_EPI_BETA) v += p.beta * sv;
  if (!rowok) v = 0.f;
  return v;
}

// Compile-time epilogues for the common flag sets (the denoiser products, heads.py deno_conv:
// conv+bias+ReLU, conv+bias+residual forward, conv*alpha with dReLU, conv+residual backward; and
// plain / bias-only products).  The generic epi_apply tests every flag per element; at 48
// elements per lane per tile that flag walk, not HBM, bounded the skinny HBM-shaped kernels.
// Row masks, STORE_PRE, dropout, MSE, SiLU, BETA keep the generic path.  EMODE 0 = generic.
// SILU_DROP: Conformer FFN up-projection (bias, SiLU, optional dropout, optional STORE_PRE);
// DROP_RESID: FFN down / attention out / conv pw2 (bias, dropout, scaled residual).  Same
// arithmetic and dropout index as epi_apply.
// MSE: the flow-matching loss head (bias, diff = v - R, loss partial, rscale * diff), same as epi_apply.
enum { SKC_EPI_GENERIC = 0, SKC_EPI_RELU = 1, SKC_EPI_RESID = 2, SKC_EPI_DRELU = 3, SKC_EPI_NONE = 4,
       SKC_EPI_SILU_DROP = 5, SKC_EPI_DROP_RESID = 6, SKC_EPI_MSE = 7 };

template <int EMODE>
__device__ __forceinline__ float skc_epi(const GemmP& p, int64_t m, int64_t n, float v, float bn, float sv, bool rowok,
                                         uint64_t seed, float keep_scale, float& mse_part, float& pre,
                                         int64_t bz = 0) {
  if constexpr (EMODE == SKC_EPI_GENERIC) {
    return epi_apply(p, bz, m, n, v, bn, sv, rowok, seed, keep_scale, mse_part, pre);
  } else {
    v += bn;  // bn is 0 without KDFM_EPI_BIAS
    if constexpr (EMODE == SKC_EPI_RELU) return fmaxf(v, 0.f);
    if constexpr (EMODE == SKC_EPI_RESID) return sv + p.rscale * v;
    if constexpr (EMODE == SKC_EPI_DRELU) return sv > 0.f ? v : 0.f;
    if constexpr (EMODE == SKC_EPI_MSE) {
      const float diff = v - sv;
      mse_part += diff * diff;
      return p.rscale * diff;
    }
    if constexpr (EMODE == SKC_EPI_SILU_DROP || EMODE == SKC_EPI_DROP_RESID) {
      pre = v;
      if constexpr (EMODE == SKC_EPI_SILU_DROP) v = siluf_(v);
      if (p.epi & KDFM_EPI_DROPOUT) {
        const uint64_t idx = ((uint64_t)bz * (uint64_t)p.M + (uint64_t)m) * (uint64_t)p.N + (uint64_t)n;
        v = dropout_keep(seed, p.rng_stream, idx, p.dropout_p) ? v * keep_scale : 0.f;
      }
      if constexpr (EMODE == SKC_EPI_DROP_RESID) v = sv + p.rscale * v;
      return v;
    }
    return v;  // SKC_EPI_NONE
  }
}

__host__ inline int skc_epi_mode(int epi) {
  switch (epi & ~KDFM_EPI_BIAS) {
    case 0: return SKC_EPI_NONE;
    case KDFM_EPI_RELU: return SKC_EPI_RELU;
    case KDFM_EPI_RESID: return SKC_EPI_RESID;
    case KDFM_EPI_DRELU: return SKC_EPI_DRELU;
    case KDFM_EPI_RESID | KDFM_EPI_DROPOUT: return SKC_EPI_DROP_RESID;
    case KDFM_EPI_MSE: return SKC_EPI_MSE;
    default: break;
  }
  if ((epi & ~(KDFM_EPI_BIAS | KDFM_EPI_DROPOUT | KDFM_EPI_STORE_PRE)) == KDFM_EPI_SILU) return SKC_EPI_SILU_DROP;
  return SKC_EPI_GENERIC;
}

// Row-stream / wide-tile entry points (rowstream.hip).  try_* return -1 when the descriptor is
// not eligible (caller falls back to the generic kernel), else a kdfm_status.
int try_rowstream_fwd(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st);
int try_rowstream_wgrad(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st);
int64_t rowstream_wgrad_ws(const GemmP& p, int amode, int bmode, int64_t batch);
// C(m,n) += alpha * sum_{s<S} ws[s][m][n] in slab order (n == ones_col -> ones_out[m]); one thread
// per element sums all S partials when `ordered` (deterministic mode), else slabs of 16.
int launch_split_fold(const GemmP& p, int64_t S, bool ordered, hipStream_t st);
// Row-parallel weight gradient with ordered fold (wgrad.hip); -1 when not eligible.
int try_wgrad_rows(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st);
int64_t wgrad_rows_ws(const GemmP& p, int amode, int bmode, int64_t batch);
// Weight-stationary skinny forward (skinny.hip); -1 when not eligible.
int try_skinny_fwd(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st);

}  // namespace kdfm
