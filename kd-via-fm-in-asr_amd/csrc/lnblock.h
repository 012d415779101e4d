// Building blocks of the LayerNorm-fused Conformer sub-block kernels (ffn.hip: macaron FFN;
// lnproj.hip: attention q|k|v projection and conv-module pointwise conv + GLU).
//
// All of them compute transposed products C^T (32 features x 32 rows) = W (32 x K) x X^T with
// v_mfma_f32_32x32x16_bf16: the A operand is a fragment of a prepared, fragment-major weight image
// (one lane-contiguous 1 KB block per (32-row tile, 16-wide k-step): conflict-free ds_read_b128),
// staged through LDS and shared by the waves of a workgroup; the B operand is the wave's rows, lane
// (r, h) holding the 8 features 16 ks + 8 h .. +7 of row r.  The accumulator gives lane (r, h) the
// features 8 q + 4 h + 0..3 of row r; one v_permlane32_swap per packed bf16 dword turns such a tile
// into the B operand of a following product (cdna_hip_programming.md T21).
#pragma once
#include "gemm_common.h"

namespace kdfm {
namespace lnb {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

constexpr int FRAG_U4 = 64;       // uint4 (8 bf16) units per fragment: one per lane

__device__ __forceinline__ bf16x8 as_bf(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ f32x16 mfma32(const uint4& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(a), b, c, 0, 0, 0);
}

__device__ __forceinline__ void swap_halves(uint32_t& a, uint32_t& b) {
  // lanes 32-63 of a <-> lanes 0-31 of b
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

// pk[q] = packed bf16 of the accumulator features 8 q + 4 h + 0..3 -> B operands of the two 16-wide
// k-steps of the tile (lanes 0-31: k 0..7, lanes 32-63: k 8..15)
__device__ __forceinline__ void tile_operands(uint32_t (&pk)[4][2], bf16x8 (&b)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    swap_halves(pk[2 * s][0], pk[2 * s + 1][0]);
    swap_halves(pk[2 * s][1], pk[2 * s + 1][1]);
    b[s] = __builtin_bit_cast(bf16x8, u32x4v{pk[2 * s][0], pk[2 * s][1], pk[2 * s + 1][0], pk[2 * s + 1][1]});
  }
}

__device__ __forceinline__ void pack4(uint32_t (&pk)[2], const float (&v)[4]) {
  pk[0] = pack_bf16x2(v[0], v[1]);
  pk[1] = pack_bf16x2(v[2], v[3]);
}

// Double-buffered staging of weight-image blocks into LDS.  Iteration `it` stages SLOTS blocks of SF
// fragments: block (SLOTS it + slot) starts at fragment ((SLOTS it + slot) * STRIDE + OFF) of the
// image (blocks >= nblk are zero-filled).  All of a stage's global loads are issued before its LDS
// stores (registers carry the next stage while the current one computes).
template <int SF, int OFF, int STRIDE, int SLOTS, int NT>
struct Stager {
  static constexpr int UNITS = SLOTS * SF * FRAG_U4;
  static constexpr int PER = (UNITS + NT - 1) / NT;
  uint4 pre[PER];
  __device__ __forceinline__ void load(const uint4* __restrict__ img, int it, int nblk) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int u = threadIdx.x + NT * i;
      const int slot = u / (SF * FRAG_U4), w = u - slot * SF * FRAG_U4;
      const int c = SLOTS * it + slot;
      pre[i] = (u < UNITS && c < nblk) ? img[((int64_t)c * STRIDE + OFF) * FRAG_U4 + w] : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(uint4* lds, int buf) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int u = threadIdx.x + NT * i;
      if (u < UNITS) lds[buf * UNITS + u] = pre[i];
    }
  }
  // this slot's block of the stage in buffer `buf`
  __device__ __forceinline__ static const uint4* block(const uint4* lds, int buf, int slot) {
    return lds + buf * UNITS + slot * SF * FRAG_U4;
  }
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gl_void_t;

// The same double-buffered staging by LDS-DMA (global_load_lds_dwordx4): one wave-instruction moves
// one 1 KB fragment of the image (lane l: bytes 16 l .. 16 l + 15) straight into its LDS block, so no
// staging registers and no ds_write pass.  A slot past the last block gets the last block again
// (finite data for callers that compute on it branch-free and discard the result).  The DMA of a stage is retired by the vmcnt(0) that the next __syncthreads()
// emits while an LDS-DMA is in flight (cdna_hip_programming.md §5 'Async global->LDS copy').
template <int SF, int OFF, int STRIDE, int SLOTS, int NT>
struct DmaStager {
  static constexpr int UNITS = SLOTS * SF * FRAG_U4;
  static constexpr int NFR = SLOTS * SF;
  static constexpr int NW = NT / 64;
  __device__ __forceinline__ static void issue(const uint4* __restrict__ img, int it, int nblk, uint4* lds, int buf) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < (NFR + NW - 1) / NW; ++i) {
      const int f = wave + NW * i;   // wave-uniform
      if (f < NFR) {
        const int slot = f / SF, w = f - slot * SF;
        const int c = SLOTS * it + slot < nblk ? SLOTS * it + slot : nblk - 1;
        __builtin_amdgcn_global_load_lds((gl_void_t*)(img + ((int64_t)c * STRIDE + OFF + w) * FRAG_U4 + lane),
                                         (lds_void_t*)(lds + buf * UNITS + f * FRAG_U4), 16, 0, 0);
      }
    }
  }
  __device__ __forceinline__ static const uint4* block(const uint4* lds, int buf, int slot) {
    return lds + buf * UNITS + slot * SF * FRAG_U4;
  }
};

// Workgroup barrier that retires this wave's LDS-DMA stage and its LDS reads but leaves its N youngest
// vector-memory operations -- the side-output stores issued after the stage's DMA -- in flight.  Loads,
// stores and LDS-DMA retire in issue order on one counter (MI355X_MICROARCH.md 'vmcnt'), so vmcnt(N)
// with the N stores issued after the DMA guarantees the DMA has landed; a __syncthreads() there waits
// vmcnt(0) and drains the stores too.  Encoding (gfx9 s_waitcnt): vmcnt bits [3:0] + [15:14],
// expcnt [6:4] (7 = no wait), lgkmcnt [11:8] (0).
template <int N>
__device__ __forceinline__ void dma_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
  __builtin_amdgcn_s_barrier();
}

// dst[0, na) = a[0, na), dst[na, na + nb) = b[0, nb) in LDS (bias tables): every thread issues all of
// its (at most MAXE) loads at clamped addresses first and writes LDS afterwards -- a fill loop with a
// load per iteration waits for each load in turn (vmcnt(0) per element)
template <int MAXE, int NT>
__device__ __forceinline__ void fill_vec3(float* dst, const float* __restrict__ a, int na, const float* __restrict__ b,
                                          int nb, const float* __restrict__ c, int nc) {
  constexpr int PER = (MAXE + NT - 1) / NT;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = (int)threadIdx.x + i * NT;
    const float* src = e < na ? a + e : (e < na + nb ? b + (e - na) : (e < na + nb + nc ? c + (e - na - nb) : a));
    v[i] = *src;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = (int)threadIdx.x + i * NT;
    if (e < na + nb + nc) dst[e] = v[i];
  }
}
template <int MAXE, int NT>
__device__ __forceinline__ void fill_vec2(float* dst, const float* __restrict__ a, int na, const float* __restrict__ b,
                                          int nb) {
  fill_vec3<MAXE, NT>(dst, a, na, b, nb, a, 0);
}
// up to six sources (bias tables followed by LayerNorm gamma / beta)
template <int MAXE, int NT>
__device__ __forceinline__ void fill_vec6(float* dst, const float* a, int na, const float* b, int nb, const float* c,
                                          int nc, const float* e4, int n4, const float* e5, int n5, const float* e6,
                                          int n6) {
  constexpr int PER = (MAXE + NT - 1) / NT;
  const int o1 = na, o2 = na + nb, o3 = o2 + nc, o4 = o3 + n4, o5 = o4 + n5, o6 = o5 + n6;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = (int)threadIdx.x + i * NT;
    const float* src = e < o1 ? a + e
                     : e < o2 ? b + (e - o1)
                     : e < o3 ? c + (e - o2)
                     : e < o4 ? e4 + (e - o3)
                     : e < o5 ? e5 + (e - o4)
                     : e < o6 ? e6 + (e - o5) : a;
    v[i] = *src;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = (int)threadIdx.x + i * NT;
    if (e < o6) dst[e] = v[i];
  }
}
template <int MAXE, int NT>
__device__ __forceinline__ void fill_vec5(float* dst, const float* a, int na, const float* b, int nb, const float* c,
                                          int nc, const float* e4, int n4, const float* e5, int n5) {
  fill_vec6<MAXE, NT>(dst, a, na, b, nb, c, nc, e4, n4, e5, n5, a, 0);
}

// LayerNorm operands in two parts so the row loads can be issued before a barrier and the statistics /
// normalisation computed after it (gamma / beta then read from an LDS table).  Out-of-range elements are
// loaded from a clamped valid address and zeroed by a 0 / 1 multiply, not a select: with
// `in ? f(load) : 0` the compiler sinks each load into a branch and waits for it there (vmcnt(0) per
// 16-feature step: a serial chain of L2 round trips in every kernel's prologue).
template <int KS1>
__device__ __forceinline__ void ln_load(const float* __restrict__ x, int64_t row, bool ok, int d, int h,
                                        float (&xv)[KS1][8]) {
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const int k0 = ks * 16 + 8 * h;
    const bool in = ok && k0 < d;
    const float4* p = reinterpret_cast<const float4*>(x + (in ? row * d + k0 : 0));
    const float4 u = p[0], w = p[1];
    const float m = in ? 1.f : 0.f;
    xv[ks][0] = u.x * m; xv[ks][1] = u.y * m; xv[ks][2] = u.z * m; xv[ks][3] = u.w * m;
    xv[ks][4] = w.x * m; xv[ks][5] = w.y * m; xv[ks][6] = w.z * m; xv[ks][7] = w.w * m;
  }
}

// statistics (unless have_stats) and the bf16 B operands bx[ks] of LN(x); g / b: gamma / beta (global or
// LDS); ln_out: optional bf16 copy of the row
template <int KS1>
__device__ __forceinline__ void ln_finish(const float (&xv)[KS1][8], const float* g, const float* b, int64_t row,
                                          bool ok, int d, int h, float eps, bool have_stats, float& mean, float& rstd,
                                          bf16x8 (&bx)[KS1], uint16_t* ln_out) {
  if (!have_stats) {
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += xv[ks][j];
    s += __shfl_xor(s, 32, 64);
    mean = s / d;
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const bool in = ks * 16 + 8 * h < d;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = in ? xv[ks][j] - mean : 0.f;
        q += t * t;
      }
    }
    q += __shfl_xor(q, 32, 64);
    rstd = rsqrtf(q / d + eps);
  }
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const int k0 = ks * 16 + 8 * h;
    const bool in = k0 < d;
    const int kc = in ? k0 : 0;
    const float m = in ? 1.f : 0.f;
    const float4 g0 = *reinterpret_cast<const float4*>(g + kc), g1 = *reinterpret_cast<const float4*>(g + kc + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(b + kc), b1 = *reinterpret_cast<const float4*>(b + kc + 4);
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    float y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = ((xv[ks][j] - mean) * rstd * gg[j] + bb[j]) * m;
    bx[ks] = pack_bf16x8<bf16x8>(y);
    if (ln_out && ok && in) *reinterpret_cast<bf16x8*>(ln_out + row * d + k0) = bx[ks];
  }
}

// Row r = `row` of x (d features, 16-B aligned rows) normalised into the B operands bx[ks]
// (features 16 ks + 8 h .. +7; zero beyond d).  have_stats: mean / rstd given (backward recompute);
// else computed (two-pass, biased variance, as kdfm_layernorm_fwd).  ln_out: bf16 copy of the row.
template <int KS1>
__device__ __forceinline__ void ln_operands(const float* __restrict__ x, const float* __restrict__ g,
                                            const float* __restrict__ b, int64_t row, bool ok, int d, int h,
                                            float eps, bool have_stats, float& mean, float& rstd,
                                            bf16x8 (&bx)[KS1], uint16_t* ln_out) {
  float xv[KS1][8];
  ln_load<KS1>(x, row, ok, d, h, xv);
  ln_finish<KS1>(xv, g, b, row, ok, d, h, eps, have_stats, mean, rstd, bx, ln_out);
}

// in-register reduce-scatter of N values over the 16 lanes of a DPP row (lane bits 8,4,2,1): afterwards
// lane (b8 b4 b2 b1) holds the 16-lane sums of the original entries b8 N/2 + b4 N/4 + b2 N/8 + b1 N/16 + j
template <int N, int M>
__device__ __forceinline__ void rs_step(const float (&in)[N], float (&out)[N / 2], int lane) {
  const bool up = (lane & M) != 0;
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    const float send = up ? in[j] : in[j + N / 2];
    const float keep = up ? in[j + N / 2] : in[j];
    out[j] = keep + __shfl_xor(send, M, 64);
  }
}

// LayerNorm backward of the lane's row from dln in the accumulator layout (dl[mt*16 + 4q + i] =
// feature mt*32 + 8q + 4h + i): dx = rstd (g dln - mean(g dln) - xhat mean(g dln xhat)) + dres, and
// the dgamma (sum dln xhat) / dbeta (sum dln) partials of the lane's 16-row group written to
// part[grp][2d] (the kdfm_layernorm_bwd_part layout, folded by kdfm_ln_fold).  Every lane of the
// wave must call it (cross-lane reductions); row_base = first row of the wave's 32-row tile.
template <int DT>
__device__ __forceinline__ void ln_backward_rows(const float (&dl)[DT * 16], const float* __restrict__ x,
                                                 const float* __restrict__ g, const float* __restrict__ dres,
                                                 float* __restrict__ dx, float* __restrict__ part, int64_t nparts,
                                                 int64_t row_base, int64_t row, bool ok, int d, float mean,
                                                 float rstd, int lane) {
  constexpr int NV = DT * 16;
  const int h = lane >> 5;
  // loads are issued in two batches, each before any store and consumed as a batch (x and gamma, then
  // the residual-gradient rows): a load under a condition, or issued after this function's own stores,
  // is waited for one at a time; two batches keep the live registers of 2-wave-per-SIMD kernels in bounds
  float xh[NV], gy[NV];
  float s1 = 0.f, s2 = 0.f;
  {
    float4 xr[DT][4], gq[DT][4];
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = mt * 32 + 8 * q + 4 * h;
        const bool in = ok && n0 < d;
        xr[mt][q] = *reinterpret_cast<const float4*>(x + (in ? row * d + n0 : 0));
        gq[mt][q] = *reinterpret_cast<const float4*>(g + (n0 < d ? n0 : 0));
      }
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = mt * 32 + 8 * q + 4 * h;
        const float m = (ok && n0 < d) ? 1.f : 0.f;
        const float xv[4] = {xr[mt][q].x, xr[mt][q].y, xr[mt][q].z, xr[mt][q].w};
        const float gv[4] = {gq[mt][q].x, gq[mt][q].y, gq[mt][q].z, gq[mt][q].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = mt * 16 + 4 * q + i;
          const float xhat = (xv[i] - mean) * rstd * m;
          xh[e] = xhat;
          gy[e] = dl[e] * gv[i] * m;
          s1 += gy[e];
          s2 += gy[e] * xhat;
        }
      }
  }
  float4 dr[DT][4];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = mt * 32 + 8 * q + 4 * h;
      const bool in = ok && n0 < d;
      dr[mt][q] = *reinterpret_cast<const float4*>(dres + (in ? row * d + n0 : 0));
    }
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  s1 /= d;
  s2 /= d;
  if (ok) {
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = mt * 32 + 8 * q + 4 * h;
        if (n0 >= d) continue;
        const float rv[4] = {dr[mt][q].x, dr[mt][q].y, dr[mt][q].z, dr[mt][q].w};
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = mt * 16 + 4 * q + i;
          o[i] = rstd * (gy[e] - s1 - xh[e] * s2) + rv[i];
        }
        *reinterpret_cast<float4*>(dx + row * d + n0) = make_float4(o[0], o[1], o[2], o[3]);
      }
  }
  const int64_t grp = row_base / 16 + ((lane >> 4) & 1);
  const int base = ((lane & 8) ? NV / 2 : 0) + ((lane & 4) ? NV / 4 : 0) + ((lane & 2) ? NV / 8 : 0) +
                   ((lane & 1) ? NV / 16 : 0);
  float* pr = part + grp * 2 * d;
#pragma unroll
  for (int qty = 0; qty < 2; ++qty) {
    float v0[NV], r1[NV / 2], r2[NV / 4], r3[NV / 8], r4[NV / 16];
#pragma unroll
    for (int e = 0; e < NV; ++e) v0[e] = ok ? (qty == 0 ? dl[e] * xh[e] : dl[e]) : 0.f;
    rs_step<NV, 8>(v0, r1, lane);
    rs_step<NV / 2, 4>(r1, r2, lane);
    rs_step<NV / 4, 2>(r2, r3, lane);
    rs_step<NV / 8, 1>(r3, r4, lane);
    if (grp < nparts) {
#pragma unroll
      for (int j = 0; j < NV / 16; ++j) {
        const int e = base + j;
        const int n = (e / 16) * 32 + 8 * ((e % 16) / 4) + 4 * h + (e % 4);
        if (n < d) pr[qty * d + n] = r4[j];
      }
    }
  }
}

// d -> (KS1 = 16-wide k-steps over d, DT = 32-wide feature tiles over d) of the compiled variants
__host__ __device__ inline int ln_dims(int64_t d, int& KS1, int& DT) {
  if (d % 8 != 0) return -1;
  if (d > 80 && d <= 96) { KS1 = 6; DT = 3; return 0; }
  if (d > 160 && d <= 176) { KS1 = 11; DT = 6; return 0; }
  if (d > 176 && d <= 192) { KS1 = 12; DT = 6; return 0; }
  return -1;
}

inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

}  // namespace lnb
}  // namespace kdfm
