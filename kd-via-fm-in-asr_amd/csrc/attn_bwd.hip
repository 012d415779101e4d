// Fused relative-position multi-head attention backward (bf16 MFMA 16x16x32, f32 accumulate).
//
// NeMo RelPositionMultiHeadAttention (Appendix A.7; per ConformerLayer, conformer_encoder.py:685-692):
//   S = (Qu K^T + rel_shift(Qv Ppos^T)) * scale, P = masked softmax(S), Pd = dropout(P), O = Pd V
// with rel_shift as the index map bd[i][j] = Qv_i . Ppos[T-1-i+j].  Given dO and the forward's
// saved P, the gradients are
//   dP = dropout'(dO V^T),  r_i = sum_j dP P,  dS = P (dP - r_i) scale
//   dQu = dS K,  dQv_i = sum_j dS[i][j] Ppos[T-1-i+j],  dK = dS^T Qu,  dV = Pd^T dO,
//   dPpos[r] = sum_{b, i} dS[i][r-(T-1)+i] Qv_i.
// The unfused path materialised dPd, dAC (B,H,T,T) and dBD (B,H,T,2T-1) in HBM (f32) and ran five
// batched GEMMs over them.  Here nothing of size T x T besides the saved P is read or written:
//   * the row sums r_i = sum_j dP P equal dO_i . O_i (O = Pd V: FlashAttention's D_i), one row dot
//     product over the saved forward output;
//   * kernel 1 (one workgroup per (b, h, 64 query rows)): dPd = dO V^T on the fly,
//     then dQu += dS K and dQv += skew(dS) Pband — the skew is the forward's band trick in reverse:
//     dS is written into a per-wave LDS tile at column j - i + 15 and multiplied by the 128-row
//     band of Ppos the block addresses;
//   * kernel 2 (one workgroup per (b, h, 64 keys)): dPd^T = V dO^T on the fly, P^T staged through
//     LDS from coalesced row loads, dV += Pd^T dO and dK += dS^T Qu over all query blocks;
//   * kernel 3 (one workgroup per (h, 64 relative positions, batch chunk)): dS recomputed for the
//     (i, j) diagonal band of its positions, dPpos += skew(dS)^T Qv; per-chunk partials are folded
//     in chunk order.
// The dropout mask is the forward's counter-RNG draw (same index -> same mask).  Every output
// element is owned by one workgroup and the fold is ordered: deterministic, no atomics.
#include "gemm_common.h"

namespace kdfm {
namespace {

constexpr int BQ = 64;             // query rows per workgroup (kernel 1), 4 waves x 16
constexpr int BK = 64;             // keys per block
constexpr int BDK = 64;            // head dim padded to 2 MFMA k-steps
constexpr int LR = BDK + 8;        // bf16 row stride of [row][c] tiles
constexpr int LT = 64 + 8;         // bf16 row stride of [c][64 rows] transposed tiles
constexpr int LW = 64 + 8;         // bf16 row stride of per-wave [16][64] tiles
constexpr int BANDR = 144;         // Ppos band rows staged (127 addressed, the rest zero)
constexpr int LB = BANDR + 8;      // bf16 row stride of the transposed band [c][band row]
constexpr int LG = 96 + 8;         // bf16 row stride of the per-wave skewed dS tile [16][96]
constexpr int NPQ = 32;            // query rows per step of kernel 3
constexpr int NPJ = 96;            // keys per step of kernel 3 (64 positions + 31 rows of skew)
constexpr int LDL = NPJ + 8;       // bf16 row stride of kernel 3's dS tile
constexpr int LQ3 = NPQ + 8;       // bf16 row stride of kernel 3's Qv^T tile

struct AbP {
  const float* dO; const float* qu; const float* qv; const float* k; const float* v; const float* pos; const float* P;
  const int64_t* lens;
  float* dqu; float* dqv; float* rsum; float* dk; float* dv; float* dpos_part;
  int64_t B, H, T, d, dkh, ldq, ldkv;
  float scale, p_drop;
  const uint64_t* seed; uint64_t rng_stream;
  int bpc;   // batches per chunk (kernel 3)
};

__device__ __forceinline__ bf16x8 frag8(const float* src, int valid) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  if (valid >= 4) a = *reinterpret_cast<const float4*>(src);
  if (valid >= 8) b = *reinterpret_cast<const float4*>(src + 4);
  const float t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return pack_bf16x8<bf16x8>(t);
}

__device__ __forceinline__ void st4(uint16_t* dst, float4 v) {
  const uint32_t lo = pack_bf16x2(v.x, v.y);
  const uint32_t hi = pack_bf16x2(v.z, v.w);
  *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
}

__device__ __forceinline__ void wsync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float g16_sum(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// rows [r0, r0 + n) of a (rows, ld) f32 matrix, columns [c0, c0 + dk) -> bf16 [row][c] (stride LR) and/or
// [c][row] (stride ldt); rows outside [lo, hi) are zero.  256 threads.
__device__ void stage_rows(uint16_t* rc, uint16_t* cr, int ldt, const float* src, int64_t ld, int64_t base_row,
                           int r0, int n, int lo, int hi, int64_t c0, int dk) {
  const int cq = dk >> 2;
  for (int e = threadIdx.x; e < n * cq; e += 256) {
    const int rr = e / cq, c4 = (e - rr * cq) * 4;
    const int r = r0 + rr;
    const bool ok = r >= lo && r < hi;
    const float4 v = ok ? *reinterpret_cast<const float4*>(src + (base_row + r) * ld + c0 + c4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    if (rc) st4(rc + rr * LR + c4, v);
    if (cr) {
      cr[(c4 + 0) * ldt + rr] = f2bf(v.x);
      cr[(c4 + 1) * ldt + rr] = f2bf(v.y);
      cr[(c4 + 2) * ldt + rr] = f2bf(v.z);
      cr[(c4 + 3) * ldt + rr] = f2bf(v.w);
    }
  }
}

// Software-pipelined staging: fetch_rows issues the global loads of rows [r0, r0 + n) into registers
// (MAXI float4 per thread) one block ahead, put_rows writes them to the LDS tiles after the barrier
// that retires the current block, so the loads' latency hides behind the current block's MFMAs.
template <int MAXI>
__device__ __forceinline__ void fetch_rows(float4 (&v)[MAXI], const float* src, int64_t ld, int64_t base_row, int r0,
                                           int n, int lo, int hi, int64_t c0, int dk) {
  const int cq = dk >> 2;
#pragma unroll
  for (int it = 0; it < MAXI; ++it) {
    const int e = threadIdx.x + it * 256;
    const int rr = e / cq, c4 = (e - rr * cq) * 4;
    const int r = r0 + rr;
    const bool ok = e < n * cq && r >= lo && r < hi;
    v[it] = ok ? *reinterpret_cast<const float4*>(src + (base_row + r) * ld + c0 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int MAXI>
__device__ __forceinline__ void put_rows(uint16_t* rc, uint16_t* cr, int ldt, const float4 (&v)[MAXI], int n, int dk) {
  const int cq = dk >> 2;
#pragma unroll
  for (int it = 0; it < MAXI; ++it) {
    const int e = threadIdx.x + it * 256;
    if (e >= n * cq) continue;
    const int rr = e / cq, c4 = (e - rr * cq) * 4;
    if (rc) st4(rc + rr * LR + c4, v[it]);
    if (cr) {
      cr[(c4 + 0) * ldt + rr] = f2bf(v[it].x);
      cr[(c4 + 1) * ldt + rr] = f2bf(v[it].y);
      cr[(c4 + 2) * ldt + rr] = f2bf(v[it].z);
      cr[(c4 + 3) * ldt + rr] = f2bf(v[it].w);
    }
  }
}

// r[(b*H + h)*T + i] = sum_c dO[b*T + i][h*dk + c] * O[b*T + i][h*dk + c]; one wave per (row, head)
__global__ __launch_bounds__(256) void attn_rowdot_kernel(const float* __restrict__ dO, const float* __restrict__ O,
                                                          float* __restrict__ r, int64_t B, int64_t H, int64_t T,
                                                          int64_t d, int dk) {
  const int lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // (b, i, h) with h fastest
  if (e >= B * T * H) return;
  const int64_t h = e % H, bi = e / H;
  const int64_t b = bi / T, i = bi - b * T;
  float v = lane < dk ? dO[bi * d + h * dk + lane] * O[bi * d + h * dk + lane] : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) r[(b * H + h) * T + i] = v;
}

// ---------------------------------------------------------------------------------------------
// kernel 1: dQu, dQv
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AbP p) {
  __shared__ __attribute__((aligned(16))) uint16_t Vs[BK * LR];     // V block [key][c]
  __shared__ __attribute__((aligned(16))) uint16_t Kt[BDK * LT];    // K block^T [c][key]
  __shared__ __attribute__((aligned(16))) uint16_t Pbt[BDK * LB];   // Ppos band^T [c][band row]
  __shared__ __attribute__((aligned(16))) uint16_t Ds[4][16 * LW];  // per wave dS [ii][jj]
  __shared__ __attribute__((aligned(16))) uint16_t Gs[4][16 * LG];  // per wave skewed dS [ii][jj - ii + 15]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const Blk3 blk = xcd_block3();
  const int64_t bh = blk.y;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int i0 = (int)blk.x * BQ;
  const int len = p.lens ? (int)min<int64_t>(p.lens[b], p.T) : T;
  const int nkb = (len + BK - 1) / BK;
  const int npos = 2 * T - 1;
  const int64_t hoff = h * p.dkh;
  // zero padding columns / rows that staging never writes
  for (int e = threadIdx.x; e < BK * (BDK - dk); e += 256) Vs[(e / (BDK - dk)) * LR + dk + e % (BDK - dk)] = 0;
  for (int e = threadIdx.x; e < (BDK - dk) * LT; e += 256) Kt[dk * LT + e] = 0;
  for (int e = threadIdx.x; e < BDK * LB; e += 256) Pbt[e] = 0;

  const int iq = i0 + w * 16 + (lane & 15);   // A-fragment row
  bf16x8 fdo[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c0 = ks * 32 + 8 * (lane >> 4);
    fdo[ks] = frag8(p.dO + (b * p.T + (iq < T ? iq : 0)) * p.ldq + hoff + c0, iq < T ? dk - c0 : 0);
  }
  const int ib = i0 + w * 16 + 4 * (lane >> 4);   // C-layout rows ib + r
  const int64_t prow0 = (bh * p.T + ib) * p.T;
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const float keep = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;

  auto dpd = [&](f32x4 (&a)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vs + (16 * t + (lane & 15)) * LR + ks * 32 + 8 * (lane >> 4));
        a[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fdo[ks], vb, a[t], 0, 0, 0);
      }
  };

  // r_i = sum_j dP P = dO_i . O_i (attn_rowdot_kernel, before this kernel)
  float rs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rs[r] = (ib + r < T) ? p.rsum[bh * p.T + ib + r] : 0.f;

  // next key block's operands in registers: V, K rows, the Ppos band, this lane's 16 P elements
  float4 nv[3], nk[3], nb[6];
  float np[4][4];
  auto fetch = [&](int kb) {
    const int j0 = kb * BK;
    const int rbase = T - 1 - (i0 + BQ - 1) + j0;
    fetch_rows<3>(nv, p.v, p.ldkv, b * p.T, j0, BK, 0, len, hoff, dk);
    fetch_rows<3>(nk, p.k, p.ldkv, b * p.T, j0, BK, 0, len, hoff, dk);
    fetch_rows<6>(nb, p.pos, p.d, 0, rbase, 127, 0, npos, hoff, dk);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ib + r, j = j0 + 16 * t + (lane & 15);
        np[t][r] = (i < T && j < len) ? p.P[prow0 + (int64_t)r * p.T + j] : 0.f;
      }
  };

  // ---- dQu += dS K, dQv += skew(dS) Pband ----
  f32x4 aq[3], av[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) { aq[u] = f32x4{0.f, 0.f, 0.f, 0.f}; av[u] = aq[u]; }
  const int wb = 48 - 16 * w;   // this wave's band offset
  uint16_t* D = Ds[w];
  uint16_t* G = Gs[w];
  if (nkb > 0) fetch(0);
  for (int kb = 0; kb < nkb; ++kb) {
    const int j0 = kb * BK;
    __syncthreads();
    put_rows<3>(Vs, nullptr, 0, nv, BK, dk);
    put_rows<3>(nullptr, Kt, LT, nk, BK, dk);
    put_rows<6>(nullptr, Pbt, LB, nb, 127, dk);
    for (int e = lane; e < 16 * LG / 2; e += 64) reinterpret_cast<uint32_t*>(G)[e] = 0u;
    __syncthreads();
    f32x4 a[4];
    dpd(a);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = ib + r, j = j0 + 16 * t + (lane & 15);
        float g = 0.f;
        if (i < T && j < len) {
          g = a[t][r];
          if (p.p_drop > 0.f)
            g = dropout_keep(seed, p.rng_stream, (uint64_t)(prow0 + (int64_t)r * p.T + j), p.p_drop) ? g * keep : 0.f;
        }
        const float ds = np[t][r] * (g - rs[r]) * p.scale;
        const int ii = 4 * (lane >> 4) + r, jj = 16 * t + (lane & 15);
        const uint16_t bv = f2bf(ds);
        D[ii * LW + jj] = bv;
        G[ii * LG + jj - ii + 15] = bv;
      }
    if (kb + 1 < nkb) fetch(kb + 1);   // the P elements are consumed: the next block's loads overlap the MFMAs
    wsync();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 da = *reinterpret_cast<const bf16x8*>(D + (lane & 15) * LW + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const bf16x8 kbf = *reinterpret_cast<const bf16x8*>(Kt + (16 * u + (lane & 15)) * LT + ks * 32 + 8 * (lane >> 4));
        aq[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, kbf, aq[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const bf16x8 ga = *reinterpret_cast<const bf16x8*>(G + (lane & 15) * LG + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const bf16x8 pb =
            *reinterpret_cast<const bf16x8*>(Pbt + (16 * u + (lane & 15)) * LB + wb + ks * 32 + 8 * (lane >> 4));
        av[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, pb, av[u], 0, 0, 0);
      }
    }
    wsync();
  }
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r, c = 16 * u + (lane & 15);
      if (i < T && c < dk) {
        const int64_t off = (b * p.T + i) * p.ldq + hoff + c;
        p.dqu[off] = aq[u][r];
        p.dqv[off] = av[u][r];
      }
    }
}

// ---------------------------------------------------------------------------------------------
// kernel 2: dK, dV
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_kernel(AbP p) {
  __shared__ __attribute__((aligned(16))) uint16_t Os[BQ * LR];     // dO block [query][c]
  __shared__ __attribute__((aligned(16))) uint16_t Ot[BDK * LT];    // dO block^T [c][query]
  __shared__ __attribute__((aligned(16))) uint16_t Qt[BDK * LT];    // Qu block^T [c][query]
  __shared__ __attribute__((aligned(16))) float Pt[BK * (BQ + 1)];  // P block^T [key][query]
  __shared__ __attribute__((aligned(16))) uint16_t Pw[4][16 * LW];  // per wave Pd^T [key][query]
  __shared__ __attribute__((aligned(16))) uint16_t Dw[4][16 * LW];  // per wave dS^T [key][query]
  __shared__ float Rs[BQ];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const Blk3 blk = xcd_block3();
  const int64_t bh = blk.y;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int j0 = (int)blk.x * BK;
  const int len = p.lens ? (int)min<int64_t>(p.lens[b], p.T) : T;
  const int64_t hoff = h * p.dkh;
  for (int e = threadIdx.x; e < BQ * (BDK - dk); e += 256) Os[(e / (BDK - dk)) * LR + dk + e % (BDK - dk)] = 0;
  for (int e = threadIdx.x; e < (BDK - dk) * LT; e += 256) { Ot[dk * LT + e] = 0; Qt[dk * LT + e] = 0; }

  const int jk = j0 + w * 16 + (lane & 15);   // A-fragment row (key)
  bf16x8 fv[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c0 = ks * 32 + 8 * (lane >> 4);
    const bool ok = jk < len;
    fv[ks] = frag8(p.v + (b * p.T + (ok ? jk : 0)) * p.ldkv + hoff + c0, ok ? dk - c0 : 0);
  }
  const int jb = j0 + w * 16 + 4 * (lane >> 4);   // C-layout key rows jb + r
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const float keep = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  f32x4 adv[3], adk[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) { adv[u] = f32x4{0.f, 0.f, 0.f, 0.f}; adk[u] = adv[u]; }
  uint16_t* PW = Pw[w];
  uint16_t* DW = Dw[w];
  const int nqb = (j0 < len) ? (len + BQ - 1) / BQ : 0;   // query rows >= len have P == 0
  // next query block's operands in registers: dO and Qu rows, the P block (row-major, coalesced along
  // keys), the row sums
  float4 ndo[3], nqu[3];
  float npb[BQ * BK / 256];
  float nrs = 0.f;
  auto fetch = [&](int qb) {
    const int i0 = qb * BQ;
    fetch_rows<3>(ndo, p.dO, p.ldq, b * p.T, i0, BQ, 0, T, hoff, dk);
    fetch_rows<3>(nqu, p.qu, p.ldq, b * p.T, i0, BQ, 0, T, hoff, dk);
#pragma unroll
    for (int it = 0; it < BQ * BK / 256; ++it) {
      const int e = threadIdx.x + it * 256;
      const int ii = e / BK, kk = e - ii * BK;
      const int i = i0 + ii, j = j0 + kk;
      npb[it] = (i < T && j < T) ? p.P[(bh * p.T + i) * p.T + j] : 0.f;
    }
    if (threadIdx.x < BQ) nrs = (i0 + threadIdx.x < T) ? p.rsum[bh * p.T + i0 + threadIdx.x] : 0.f;
  };
  if (nqb > 0) fetch(0);
  for (int qb = 0; qb < nqb; ++qb) {
    const int i0 = qb * BQ;
    __syncthreads();
    put_rows<3>(Os, Ot, LT, ndo, BQ, dk);
    put_rows<3>(nullptr, Qt, LT, nqu, BQ, dk);
#pragma unroll
    for (int it = 0; it < BQ * BK / 256; ++it) {
      const int e = threadIdx.x + it * 256;
      const int ii = e / BK, kk = e - ii * BK;
      Pt[kk * (BQ + 1) + ii] = npb[it];
    }
    if (threadIdx.x < BQ) Rs[threadIdx.x] = nrs;
    __syncthreads();
    if (qb + 1 < nqb) fetch(qb + 1);
    // dPd^T = V dO^T (16 keys x 64 queries per wave)
    f32x4 a[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 ob = *reinterpret_cast<const bf16x8*>(Os + (16 * t + (lane & 15)) * LR + ks * 32 + 8 * (lane >> 4));
        a[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fv[ks], ob, a[t], 0, 0, 0);
      }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = 4 * (lane >> 4) + r, qq = 16 * t + (lane & 15);
        const int j = jb + r, i = i0 + qq;
        float pd = 0.f, ds = 0.f;
        if (j < len && i < T) {
          const float pv = Pt[(j - j0) * (BQ + 1) + qq];
          float g = a[t][r];
          pd = pv;
          if (p.p_drop > 0.f) {
            const uint64_t idx = (uint64_t)((bh * p.T + i) * p.T + j);
            const bool kp = dropout_keep(seed, p.rng_stream, idx, p.p_drop);
            g = kp ? g * keep : 0.f;
            pd = kp ? pv * keep : 0.f;
          }
          ds = pv * (g - Rs[qq]) * p.scale;
        }
        PW[kk * LW + qq] = f2bf(pd);
        DW[kk * LW + qq] = f2bf(ds);
      }
    wsync();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(PW + (lane & 15) * LW + ks * 32 + 8 * (lane >> 4));
      const bf16x8 da = *reinterpret_cast<const bf16x8*>(DW + (lane & 15) * LW + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const bf16x8 ob = *reinterpret_cast<const bf16x8*>(Ot + (16 * u + (lane & 15)) * LT + ks * 32 + 8 * (lane >> 4));
        const bf16x8 qb = *reinterpret_cast<const bf16x8*>(Qt + (16 * u + (lane & 15)) * LT + ks * 32 + 8 * (lane >> 4));
        adv[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, ob, adv[u], 0, 0, 0);
        adk[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, qb, adk[u], 0, 0, 0);
      }
    }
    wsync();
  }
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jb + r, c = 16 * u + (lane & 15);
      if (j < T && c < dk) {
        const int64_t off = (b * p.T + j) * p.ldkv + hoff + c;
        p.dv[off] = adv[u][r];
        p.dk[off] = adk[u][r];
      }
    }
}

// ---------------------------------------------------------------------------------------------
// kernel 3: per-chunk partials of dPpos
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void attn_bwd_dpos_kernel(AbP p) {
  __shared__ __attribute__((aligned(16))) uint16_t Vs[NPJ * LR];     // V rows jbase.. [key][c]
  __shared__ __attribute__((aligned(16))) uint16_t Dl[NPQ * LDL];    // dS [i - ib0][j - jbase]
  __shared__ __attribute__((aligned(16))) uint16_t Qt[BDK * LQ3];    // Qv^T [c][i - ib0]
  __shared__ float Rs[NPQ];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const int npos = 2 * T - 1;
  const Blk3 blk = xcd_block3();
  const int r0 = (int)blk.x * 64;
  const int64_t h = blk.y;
  const int64_t bchunk = blk.z;
  const int64_t hoff = h * p.dkh;
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const float keep = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  for (int e = threadIdx.x; e < NPJ * (BDK - dk); e += 256) Vs[(e / (BDK - dk)) * LR + dk + e % (BDK - dk)] = 0;
  for (int e = threadIdx.x; e < (BDK - dk) * LQ3; e += 256) Qt[dk * LQ3 + e] = 0;
  f32x4 acc[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qh = w & 1, kh = w >> 1;   // dS computation: query half, key half (48 keys)
  const int64_t b0 = bchunk * p.bpc;
  const int64_t b1 = min<int64_t>(p.B, b0 + p.bpc);
  // iterations (utterance b, query block ib0) that address a valid key for these positions
  auto ulen = [&](int64_t bb) { return p.lens ? (int)min<int64_t>(p.lens[bb], p.T) : T; };
  auto advance = [&](int64_t& bb, int& ib, int& ln) -> bool {
    ib += NPQ;
    while (bb < b1) {
      for (; ib < ln; ib += NPQ) {
        const int jb = r0 - (T - 1) + ib;
        if (!(jb + NPJ <= 0 || jb >= ln)) return true;
      }
      if (++bb >= b1) break;
      ib = 0;
      ln = ulen(bb);
      if (ib < ln) {
        const int jb = r0 - (T - 1) + ib;
        if (!(jb + NPJ <= 0 || jb >= ln)) return true;
      }
    }
    return false;
  };
  // next iteration's operands in registers (software pipeline): V rows, Qv rows, row sums, this
  // lane's dO fragments and 12 P elements
  float4 nvr[(NPJ * 12 + 255) / 256], nqr[(NPQ * 12 + 255) / 256];
  float nrs = 0.f;
  bf16x8 nfdo[2];
  float np[3][4];
  auto fetch = [&](int64_t bb, int ib, int ln) {
    const int jb = r0 - (T - 1) + ib;
    const int64_t bhh = bb * p.H + h;
    fetch_rows<(NPJ * 12 + 255) / 256>(nvr, p.v, p.ldkv, bb * p.T, jb, NPJ, 0, ln, hoff, dk);
    fetch_rows<(NPQ * 12 + 255) / 256>(nqr, p.qv, p.ldq, bb * p.T, ib, NPQ, 0, ln, hoff, dk);
    if (threadIdx.x < NPQ) nrs = (ib + (int)threadIdx.x < ln) ? p.rsum[bhh * p.T + ib + threadIdx.x] : 0.f;
    const int iq = ib + 16 * qh + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c0 = ks * 32 + 8 * (lane >> 4);
      const bool ok = iq < ln;
      nfdo[ks] = frag8(p.dO + (bb * p.T + (ok ? iq : 0)) * p.ldq + hoff + c0, ok ? dk - c0 : 0);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 16 * qh + 4 * (lane >> 4) + r, jl = 48 * kh + 16 * t + (lane & 15);
        const int i = ib + il, j = jb + jl;
        np[t][r] = (i < ln && j >= 0 && j < ln) ? p.P[(bhh * p.T + i) * p.T + j] : 0.f;
      }
  };
  int64_t b = b0;
  int ib0 = -NPQ, len = b0 < b1 ? ulen(b0) : 0;
  bool more = b0 < b1 && advance(b, ib0, len);
  if (more) fetch(b, ib0, len);
  while (more) {
    const int64_t bh = b * p.H + h;
    const int jbase = r0 - (T - 1) + ib0;
    const int cur_len = len;
    const int cur_ib0 = ib0;
    __syncthreads();
    put_rows<(NPJ * 12 + 255) / 256>(Vs, nullptr, 0, nvr, NPJ, dk);
    put_rows<(NPQ * 12 + 255) / 256>(nullptr, Qt, LQ3, nqr, NPQ, dk);
    if (threadIdx.x < NPQ) Rs[threadIdx.x] = nrs;
    const bf16x8 fdo[2] = {nfdo[0], nfdo[1]};
    __syncthreads();
    // dPd for queries ib0 + 16 qh + .., keys jbase + 48 kh + ..
    f32x4 a[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) a[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vs + (48 * kh + 16 * t + (lane & 15)) * LR + ks * 32 +
                                                             8 * (lane >> 4));
        a[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fdo[ks], vb, a[t], 0, 0, 0);
      }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 16 * qh + 4 * (lane >> 4) + r, jl = 48 * kh + 16 * t + (lane & 15);
        const int i = cur_ib0 + il, j = jbase + jl;
        float ds = 0.f;
        if (i < cur_len && j >= 0 && j < cur_len) {
          const int64_t idx = (bh * p.T + i) * p.T + j;
          float g = a[t][r];
          if (p.p_drop > 0.f) g = dropout_keep(seed, p.rng_stream, (uint64_t)idx, p.p_drop) ? g * keep : 0.f;
          ds = np[t][r] * (g - Rs[il]) * p.scale;
        }
        Dl[il * LDL + jl] = f2bf(ds);
      }
    // the P elements are consumed: the next iteration's loads overlap the dPpos MFMAs
    more = advance(b, ib0, len);
    if (more) fetch(b, ib0, len);
    __syncthreads();
    // dPpos[r0 + 16 w + m] += sum_i dS[i][(16 w + m) + i] Qv_i: A[m][k = i] = Dl[i][16 w + m + i]
    const int m = lane & 15, kq = 8 * (lane >> 4);
    bf16x8 fa;
#pragma unroll
    for (int e = 0; e < 8; ++e) fa[e] = (short)Dl[(kq + e) * LDL + 16 * w + m + kq + e];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const bf16x8 qb = *reinterpret_cast<const bf16x8*>(Qt + (16 * u + (lane & 15)) * LQ3 + kq);
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, qb, acc[u], 0, 0, 0);
    }
  }
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = r0 + 16 * w + 4 * (lane >> 4) + r, c = 16 * u + (lane & 15);
      if (rr < npos && c < dk) p.dpos_part[(bchunk * npos + rr) * p.d + hoff + c] = acc[u][r];
    }
}

// dpos[r][c] = sum_chunk part[chunk][r][c], chunks in order (deterministic)
__global__ __launch_bounds__(256) void attn_dpos_fold_kernel(const float* __restrict__ part, float* __restrict__ dpos,
                                                             int64_t n, int chunks) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[c * n + e];
  dpos[e] = s;
}

constexpr int DPOS_MAX_CHUNKS = 64;   // dPpos partials: one chunk per utterance (up to 64)

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_relpos_attn_bwd_ws(int64_t B, int64_t H, int64_t T, int64_t d) {
  return B * H * T + (B < kdfm::DPOS_MAX_CHUNKS ? B : (int64_t)kdfm::DPOS_MAX_CHUNKS) * (2 * T - 1) * d;
}

int kdfm_relpos_attn_bwd(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                         const float* pos, const float* P, const int64_t* lengths, float* dqu, float* dqv, float* dqkv,
                         float* dpos,
                         float* ws, int64_t ws_len, int64_t B, int64_t H, int64_t T, int64_t d, float scale,
                         float dropout_p, const uint64_t* seed, uint64_t rng_stream, void* stream) {
  return kdfm_relpos_attn_bwd_parts(dO, O, qu, qv, qkv, pos, P, lengths, dqu, dqv, dqkv, dpos, ws, ws_len, B, H, T, d,
                                    scale, dropout_p, seed, rng_stream, KDFM_ATTN_BWD_ALL, stream);
}

int kdfm_relpos_attn_bwd_parts(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                               const float* pos, const float* P, const int64_t* lengths, float* dqu, float* dqv,
                               float* dqkv, float* dpos, float* ws, int64_t ws_len, int64_t B, int64_t H, int64_t T,
                               int64_t d, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                               int32_t parts, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dO && O && qu && qv && qkv && pos && P && ws, "null pointer");
  KDFM_REQUIRE(!(parts & KDFM_ATTN_BWD_DQ) || (dqu && dqv), "dq part needs dqu / dqv");
  KDFM_REQUIRE(!(parts & KDFM_ATTN_BWD_DKV) || dqkv, "dkv part needs dqkv");
  KDFM_REQUIRE(!(parts & KDFM_ATTN_BWD_DPOS) || dpos, "dpos part needs dpos");
  KDFM_REQUIRE(H > 0 && d % H == 0, "d must be a multiple of H");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk <= 48 && dk % 4 == 0, "head dim must be a multiple of 4 and <= 48");
  KDFM_REQUIRE(T > 0 && T <= 4096 && d % 4 == 0, "bad T / d");
  KDFM_REQUIRE(dropout_p == 0.f || seed, "dropout needs a seed");
  KDFM_REQUIRE(ws_len >= kdfm_relpos_attn_bwd_ws(B, H, T, d), "workspace too small (kdfm_relpos_attn_bwd_ws)");
  KDFM_REQUIRE((((uintptr_t)dO | (uintptr_t)qu | (uintptr_t)qv | (uintptr_t)qkv | (uintptr_t)pos | (uintptr_t)P) & 15) == 0,
               "operands must be 16-byte aligned");
  if (B == 0) return KDFM_OK;
  AbP p{};
  p.dO = dO; p.qu = qu; p.qv = qv; p.k = qkv + d; p.v = qkv + 2 * d; p.pos = pos; p.P = P; p.lens = lengths;
  p.dqu = dqu; p.dqv = dqv; p.rsum = ws; p.dpos_part = ws + B * H * T;
  p.dk = dqkv ? dqkv + d : nullptr;
  p.dv = dqkv ? dqkv + 2 * d : nullptr;
  p.B = B; p.H = H; p.T = T; p.d = d; p.dkh = dk; p.ldq = d; p.ldkv = 3 * d;
  p.scale = scale; p.p_drop = dropout_p; p.seed = seed; p.rng_stream = rng_stream;
  const int chunks = (int)(B < DPOS_MAX_CHUNKS ? B : DPOS_MAX_CHUNKS);
  p.bpc = (int)ceil_div(B, chunks);
  hipStream_t st = as_stream(stream);
  int rc = KDFM_OK;
  if (parts & KDFM_ATTN_BWD_ROWDOT) {
    hipLaunchKernelGGL(attn_rowdot_kernel, dim3((unsigned)ceil_div(B * T * H, 4)), dim3(256), 0, st, dO, O, p.rsum, B,
                       H, T, d, (int)dk);
    rc = check_launch("kdfm_relpos_attn_bwd(rowdot)");
    if (rc) return rc;
  }
  if (parts & KDFM_ATTN_BWD_DQ) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((unsigned)ceil_div(T, BQ), (unsigned)(B * H)), dim3(256), 0, st, p);
    rc = check_launch("kdfm_relpos_attn_bwd(dq)");
    if (rc) return rc;
  }
  if (parts & KDFM_ATTN_BWD_DKV) {
    hipLaunchKernelGGL(attn_bwd_dkv_kernel, dim3((unsigned)ceil_div(T, BK), (unsigned)(B * H)), dim3(256), 0, st, p);
    rc = check_launch("kdfm_relpos_attn_bwd(dkv)");
    if (rc) return rc;
  }
  if (!(parts & KDFM_ATTN_BWD_DPOS)) return KDFM_OK;
  const int64_t npos = 2 * T - 1;
  hipLaunchKernelGGL(attn_bwd_dpos_kernel, dim3((unsigned)ceil_div(npos, 64), (unsigned)H, (unsigned)chunks),
                     dim3(256), 0, st, p);
  rc = check_launch("kdfm_relpos_attn_bwd(dpos)");
  if (rc) return rc;
  hipLaunchKernelGGL(attn_dpos_fold_kernel, dim3((unsigned)ceil_div(npos * d, 256)), dim3(256), 0, st, p.dpos_part,
                     dpos, npos * d, chunks);
  return check_launch("kdfm_relpos_attn_bwd(fold)");
}

}  // extern "C"
