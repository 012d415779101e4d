// Fused relative-position multi-head attention forward (bf16 MFMA, f32 softmax/accumulate).
//
// NeMo RelPositionMultiHeadAttention.forward (Appendix A.7; called per ConformerLayer,
// conformer_encoder.py:685-692): scores = ((q+u)K^T + rel_shift((q+v)P^T)) / sqrt(dk), key padding
// mask, softmax, dropout_att, P V.  The unfused path materialises AC (B,H,T,T) and BD (B,H,T,2T-1)
// in HBM; here one workgroup owns (b, h, 64 query rows) and streams 64-key blocks:
//   * S_ac = Qu K_blk^T (per wave 16 x 64), Qu/Qv fragments live in registers;
//   * the BD term only needs the 127-row band of P that the block's (i, j) pairs address
//     (r = T-1-i+j); each wave computes G = Qv P_band^T (16 x 80) and reads it back skewed from
//     LDS: S_bd[ii][jj] = G[ii][jj - ii + 15]  (rel_shift as an index map, no copy);
//   * one pass over the key blocks with an online softmax (running row max / sum, O rescaled), the
//     counter-RNG dropout mask of the unfused kernel (same index -> same mask) applied to the
//     unnormalised probabilities and O += P_drop V via MFMA (P staged through LDS into A-fragment
//     order, V staged transposed); training writes the per-row log-sum-exp lse_i = m_i + ln l_i,
//     the UNNORMALISED probabilities p~ = exp(s - m_ikb) as bf16 (B,H,T,T) and the running row max
//     m_ikb after each 64-key block (B,H,T,ceil(T/64)): P = p~ exp(m_ikb - lse_i) (the backward's
//     dK/dV and dPpos kernels read P this way: half the bytes of an f32 P, and no second pass);
//   * (the unfused backward's path) two passes: (1) row max and sum, (2) exact probabilities with
//     the P / P_drop outputs the per-op backward reads.
// Output O is written straight into the (rows, d) head-interleaved layout.
#include "gemm_common.h"
#include "attn_centre.h"

// timing probe points (tools/attn_probe.hip defines KPROBE; empty in the library)
#ifndef KPROBE
#define KPROBE(i)
#endif

namespace kdfm {
namespace {

constexpr int AQ = 64;            // query rows per workgroup (4 waves x 16)
constexpr int AKB = 64;           // keys per block
constexpr int LDVT = AKB + 8;     // bf16 row stride of V^T [c][key]
constexpr int LDPS = AKB + 8;     // bf16 row stride of the per-wave P tile [row][key]
constexpr int BAND = 128;         // P rows staged per key block (127 used)
constexpr int GW = 80;            // band columns per wave (79 used)
constexpr int LDG = GW + 1;       // f32 stride of the per-wave G tile

struct AttnP {
  const float* qu; const float* qv; const float* k; const float* v; const float* pos;
  const int64_t* lens;
  float* o; float* P; float* Pd; float* lse; uint16_t* pt; float* mblk;
  int64_t B, H, T, d, dk, ldq, ldkv;
  float scale, p_drop;
  const uint64_t* seed; uint64_t rng_stream;
};

__device__ __forceinline__ bf16x8 load_frag8(const float* head, int c0, int valid) {
  // columns c0 .. c0 + 7 of a row (head: its first column of this head) -> bf16x8, elements >= valid
  // zero (valid a multiple of 4 or >= 8); unconditional loads at a clamped column, masked by a
  // multiply (a conditional load, or a select on a loaded value, is branched around and waited for)
  const float m0 = valid >= 4 ? 1.f : 0.f, m1 = valid >= 8 ? 1.f : 0.f;
  const float4 a = *reinterpret_cast<const float4*>(head + (valid >= 4 ? c0 : 0));
  const float4 b = *reinterpret_cast<const float4*>(head + (valid >= 8 ? c0 + 4 : 0));
  const float t[8] = {a.x * m0, a.y * m0, a.z * m0, a.w * m0, b.x * m1, b.y * m1, b.z * m1, b.w * m1};
  return pack_bf16x8<bf16x8>(t);
}

__device__ __forceinline__ void store4_bf16(uint16_t* dst, float4 v) {
  const uint32_t lo = pack_bf16x2(v.x, v.y);
  const uint32_t hi = pack_bf16x2(v.z, v.w);
  *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
}

// wave-local LDS hand-off: this wave's ds_writes complete before its following ds_reads, and the
// compiler may not move LDS accesses across the point
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// reductions over the 16 lanes of a DPP row (one query row's 16 key columns of a C tile) by DPP moves
// (VALU, no LDS round trip as ds_bpermute): quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror,
// row_mirror -- every lane ends with the same value (commutative pairings of the same tree)
template <int CTRL>
__device__ __forceinline__ float dppmov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float group16_max(float v) {
  v = fmaxf(v, dppmov<0xB1>(v));
  v = fmaxf(v, dppmov<0x4E>(v));
  v = fmaxf(v, dppmov<0x141>(v));
  return fmaxf(v, dppmov<0x140>(v));
}
__device__ __forceinline__ float group16_sum(float v) {
  v += dppmov<0xB1>(v);
  v += dppmov<0x4E>(v);
  v += dppmov<0x141>(v);
  return v + dppmov<0x140>(v);
}

// NU: 16-column output tiles of the head dim (3: dk <= 48, 4: dk <= 64, 8: dk <= 128 -- FastConformer-XL's
// 1024 / 8 heads); the head dim is padded to KS MFMA k-steps of 32 (2, or 4 for NU = 8); WPT (single pass): p~ and m_blk
// are written -- through buffer stores whose out-of-range lanes carry an offset past the buffer (dropped
// by the range check) instead of a branch, so each key block issues a fixed number of stores and the
// wait for the next block's staged loads counts past them instead of draining them (vmcnt(0))
template <bool TWO_PASS, int NU, bool WPT = false>
__global__ __launch_bounds__(256, NU == 3 ? 2 : 1) void relpos_attn_fwd_kernel(AttnP p) {
  constexpr int KS = NU > 4 ? 4 : 2;   // MFMA k-steps over the padded head dim
  constexpr int DKP = 32 * KS;         // head dim padded
  constexpr int LDR = DKP + 8;         // bf16 row stride of the [row][c] tiles (K, P band)
  __shared__ __attribute__((aligned(16))) uint16_t Ks[AKB * LDR];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[DKP * LDVT];
  __shared__ __attribute__((aligned(16))) uint16_t Pr[BAND * LDR];
  __shared__ __attribute__((aligned(16))) float Gs[4][16 * LDG];
  __shared__ __attribute__((aligned(16))) uint16_t Ps[4][16 * LDPS];
  __shared__ __attribute__((aligned(16))) float Cn[2][DKP];   // key / value centre (attn_centre.h)

  KPROBE(0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dk;
  const Blk3 blk = xcd_block3();
  const int64_t bh = blk.y;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int i0 = (int)blk.x * AQ;
  const int len = p.lens ? (int)p.lens[b] : T;
  const int nkb = (min(len, T) + AKB - 1) / AKB;  // key blocks with at least one valid key
  const int npos = 2 * T - 1;
  constexpr uint32_t OOB = 0x80000000u;
  const int nkb_all = (T + AKB - 1) / AKB;
  const __amdgpu_buffer_rsrc_t rpt =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.pt, (short)0, WPT ? (int)(p.B * p.H * p.T * p.T * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rmb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.mblk, (short)0, WPT ? (int)(p.B * p.H * p.T * nkb_all * 4) : 0, 0x00020000);
  const int64_t hoff = h * p.dk;

  // zero the K / V^T / band images once with 16-byte stores (the padded head-dim columns are never
  // overwritten afterwards; the data columns are rewritten by store_stage after a barrier)
  static_assert((AKB * LDR) % 8 == 0 && (DKP * LDVT) % 8 == 0 && (BAND * LDR) % 8 == 0, "16-byte images");
  for (int e = threadIdx.x; e < AKB * LDR / 8; e += 256) reinterpret_cast<uint4*>(Ks)[e] = make_uint4(0u, 0u, 0u, 0u);
  for (int e = threadIdx.x; e < DKP * LDVT / 8; e += 256) reinterpret_cast<uint4*>(Vt)[e] = make_uint4(0u, 0u, 0u, 0u);
  for (int e = threadIdx.x; e < BAND * LDR / 8; e += 256) reinterpret_cast<uint4*>(Pr)[e] = make_uint4(0u, 0u, 0u, 0u);

  // this lane's query row (A-fragment row) and its Qu / Qv fragments
  const int iq = i0 + w * 16 + (lane & 15);
  bf16x8 fu[KS], fv[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int c0 = ks * 32 + 8 * (lane >> 4);
    const int valid = (iq < T) ? dk - c0 : 0;
    const int64_t off = (b * p.T + (iq < T ? iq : 0)) * p.ldq + hoff;
    fu[ks] = load_frag8(p.qu + off, c0, valid);
    fv[ks] = load_frag8(p.qv + off, c0, valid);
  }

  // rows owned by this lane in the C layout: ii = 4*(lane>>4) + r
  const int ib = i0 + w * 16 + 4 * (lane >> 4);
  float mrow[4], lrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mrow[r] = -3.0e38f; lrow[r] = 0.f; }

  // ---- staging of one key block: all global loads of a stage are issued before any LDS store
  // (register staging; the next block's loads are in flight while this block computes).  The per-thread
  // staging geometry is loop invariant and computed once; every load is issued unconditionally from a
  // clamped valid address and out-of-range elements are zeroed by a select at store time (a load under
  // a runtime condition is branched around and waited for one by one) ----
  constexpr int KU = (AKB * 4 * NU + 255) / 256;    // K / V float4 per thread (dk <= 16 NU)
  constexpr int PU = (BAND * 4 * NU + 255) / 256;   // P-band float4 per thread
  const int cq = dk >> 2;
  int kj[KU], kc[KU], pj[PU], pc[PU];
  uint32_t kin = 0u, pin = 0u;   // bit i: slot i maps to a real (row, column) of the tile
#pragma unroll
  for (int i = 0; i < KU; ++i) {
    const int e = threadIdx.x + i * 256;
    const bool in = e < AKB * cq;
    const int ee = in ? e : 0;
    kj[i] = ee / cq;
    kc[i] = (ee - kj[i] * cq) * 4;
    kin |= (in ? 1u : 0u) << i;
  }
#pragma unroll
  for (int i = 0; i < PU; ++i) {
    const int e = threadIdx.x + i * 256;
    const bool in = e < BAND * cq;
    const int ee = in ? e : 0;
    pj[i] = ee / cq;
    pc[i] = (ee - pj[i] * cq) * 4;
    pin |= (in ? 1u : 0u) << i;
  }
  const float* kbase = p.k + b * p.T * p.ldkv + hoff;
  const float* vbase = p.v + b * p.T * p.ldkv + hoff;
  const float* pbase = p.pos + hoff;
  // key / value centring (attn_centre.h): K and V are staged as bf16(K_j - kc) and bf16(V_j - vc); the
  // scores (hence lse, p~, m_blk) are those of the centred keys, O gets (sum_j Pd_ij) vc back in f32
  float4 rk[KU], rv[KU], rp[PU];
  uint32_t kok = 0u, pok = 0u;   // validity of the staged slots of the stage in flight
  auto load_stage = [&](int j0, bool with_v) {
    kok = 0u;
#pragma unroll
    for (int i = 0; i < KU; ++i) {
      const int j = j0 + kj[i];
      const bool ok = ((kin >> i) & 1u) && j < T;
      const int64_t off = (int64_t)(ok ? j : 0) * p.ldkv + kc[i];
      rk[i] = *reinterpret_cast<const float4*>(kbase + off);
      if (with_v) rv[i] = *reinterpret_cast<const float4*>(vbase + off);
      kok |= (ok ? 1u : 0u) << i;
    }
    const int rbase = T - 1 - (i0 + AQ - 1) + j0;  // P band rows r = rbase + rr
    pok = 0u;
#pragma unroll
    for (int i = 0; i < PU; ++i) {
      const int r = rbase + pj[i];
      const bool ok = ((pin >> i) & 1u) && r >= 0 && r < npos;
      rp[i] = *reinterpret_cast<const float4*>(pbase + (int64_t)(ok ? r : 0) * p.d + pc[i]);
      pok |= (ok ? 1u : 0u) << i;
    }
  };
  auto store_stage = [&](bool with_v) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < KU; ++i) {
      if ((kin >> i) & 1u) {
        const bool ok = (kok >> i) & 1u;
        // the centre read back from LDS (float4 copies held across the loop cost 24 VGPRs)
        const float4 ck = *reinterpret_cast<const float4*>(&Cn[0][kc[i]]);
        const float4 cv = *reinterpret_cast<const float4*>(&Cn[1][kc[i]]);
        const float4 kk = make_float4(rk[i].x - ck.x, rk[i].y - ck.y, rk[i].z - ck.z, rk[i].w - ck.w);
        store4_bf16(Ks + kj[i] * LDR + kc[i], ok ? kk : z);
        if (with_v) {
          const float4 vc = make_float4(rv[i].x - cv.x, rv[i].y - cv.y, rv[i].z - cv.z, rv[i].w - cv.w);
          const float4 vv = ok ? vc : z;
          Vt[(kc[i] + 0) * LDVT + kj[i]] = f2bf(vv.x);
          Vt[(kc[i] + 1) * LDVT + kj[i]] = f2bf(vv.y);
          Vt[(kc[i] + 2) * LDVT + kj[i]] = f2bf(vv.z);
          Vt[(kc[i] + 3) * LDVT + kj[i]] = f2bf(vv.w);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < PU; ++i)
      if ((pin >> i) & 1u) store4_bf16(Pr + pj[i] * LDR + pc[i], ((pok >> i) & 1u) ? rp[i] : z);
  };

  // scores of this wave's 16 rows x 64 keys of block j0, C layout: s[t][r] = S[ii][16t + (lane&15)]
  auto scores = [&](int j0, float (&s)[4][4]) {
    f32x4 ac[4], g[5];
#pragma unroll
    for (int t = 0; t < 4; ++t) ac[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 5; ++t) g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int wb = 48 - 16 * w;  // this wave's band offset inside Pr
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kof = ks * 32 + 8 * (lane >> 4);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 kb = *reinterpret_cast<const bf16x8*>(Ks + (16 * t + (lane & 15)) * LDR + kof);
        ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fu[ks], kb, ac[t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const bf16x8 pb = *reinterpret_cast<const bf16x8*>(Pr + (wb + 16 * t + (lane & 15)) * LDR + kof);
        g[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fv[ks], pb, g[t], 0, 0, 0);
      }
    }
    float* G = Gs[w];
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) G[(4 * (lane >> 4) + r) * LDG + 16 * t + (lane & 15)] = g[t][r];
    wave_lds_sync();
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * (lane >> 4) + r, jj = 16 * t + (lane & 15);
        const int j = j0 + jj;
        const float bd = G[ii * LDG + jj - ii + 15];
        s[t][r] = (j < len && j < T) ? (ac[t][r] + bd) * p.scale : -3.0e38f;
      }
    wave_lds_sync();  // G is rewritten by the next call
  };

  // ---- pass 1 (two-pass mode): row max / sum ----
  // (the first stage's loads are issued before the centre: they are raw rows, centred at store time)
  if (TWO_PASS && nkb > 0) load_stage(0, false);
  if (!TWO_PASS && nkb > 0) load_stage(0, true);
  kv_centre<DKP>(kbase, vbase, p.ldkv, min(len, T), dk, Cn);
  if constexpr (WPT) {
    // the loop body leaves its 4 m_blk + 16 p~ stores behind the next block's loads; the same number of
    // (range-dropped) stores behind the first block's loads lets the compiler's wait for a staged load
    // count past them on every path into the loop instead of draining the stores (vmcnt(0))
#pragma unroll
    for (int i = 0; i < 20; ++i) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)0, rpt, OOB + 2u * i, 0, 0);
  }
  for (int kb = 0; kb < (TWO_PASS ? nkb : 0); ++kb) {
    const int j0 = kb * AKB;
    __syncthreads();
    store_stage(false);
    __syncthreads();
    if (kb + 1 < nkb) load_stage(j0 + AKB, false);
    else if (nkb > 0) load_stage(0, true);  // first block of pass 2
    float s[4][4];
    scores(j0, s);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
      mx = group16_max(mx);
      const float mn = fmaxf(mrow[r], mx);
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) sum += (s[t][r] > -1.0e38f) ? __expf(s[t][r] - mn) : 0.f;
      sum = group16_sum(sum);
      lrow[r] = lrow[r] * ((mrow[r] > -1.0e38f) ? __expf(mrow[r] - mn) : 0.f) + sum;
      mrow[r] = mn;
    }
  }
  float inv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) inv[r] = TWO_PASS ? ((ib + r < len && lrow[r] > 0.f) ? 1.f / lrow[r] : 0.f) : 1.f;

  // ---- pass 2: probabilities, dropout, O += Pd V ----
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const uint64_t dkey = rng_key(seed, p.rng_stream);
  const float keep_scale = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  f32x4 oacc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) oacc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t prow0 = (bh * p.T + ib) * p.T;  // P row of (ib, j = 0)
  // per owned row: flat index of its (i, j = 0) element (dropout counter, p~ offset) and whether i < T
  int64_t prow[4];
  uint64_t dpair[4];   // attn_drop_rowpairs of the owned rows
  bool rowin[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    prow[r] = prow0 + (int64_t)r * p.T;
    dpair[r] = attn_drop_rowpairs(bh * p.T + ib + r, p.T);
    rowin[r] = ib + r < T;
  }
  const bool drop = p.p_drop > 0.f;
  float ps[4] = {0.f, 0.f, 0.f, 0.f};   // sum_j Pd_ij (dropout only; rescaled with O in the online softmax)
  KPROBE(1);
  // single pass: only the key blocks with a valid key (the p~ zeros of the first block past them are
  // written after the loop), and the next stage is always loaded (the last block reloads itself), so
  // every iteration issues the same loads and stores
  for (int kb = 0; kb < (TWO_PASS ? nkb_all : nkb); ++kb) {
    const int j0 = kb * AKB;
    const bool live = TWO_PASS ? kb < nkb : true;
    if (live) {
      __syncthreads();
      store_stage(true);
      __syncthreads();
      if (TWO_PASS) {
        if (kb + 1 < nkb) load_stage(j0 + AKB, true);
      } else {
        load_stage(kb + 1 < nkb ? j0 + AKB : j0, true);
      }
    }
    KPROBE(2 + 4 * kb);
    float s[4][4];
    if (live) {
      scores(j0, s);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[t][r] = -3.0e38f;
    }
    if (!TWO_PASS && live) {  // online softmax: rescale the running sum and O to the new row max
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float mx = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
        mx = group16_max(mx);
        const float mn = fmaxf(mrow[r], mx);
        const float corr = (mrow[r] > -1.0e38f) ? __expf(mrow[r] - mn) : 0.f;
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) sum += (s[t][r] > -1.0e38f) ? __expf(s[t][r] - mn) : 0.f;
        lrow[r] = lrow[r] * corr + group16_sum(sum);
        mrow[r] = mn;
        ps[r] *= corr;
#pragma unroll
        for (int u = 0; u < NU; ++u) oacc[u][r] *= corr;
      }
    }
    if (WPT && live) {   // the running max this block's p~ is relative to (the 16 lanes of a row hold the same)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, mrow[r]), rmb,
                                              rowin[r] ? (uint32_t)(((bh * p.T + ib + r) * nkb_all + kb) * 4) : OOB,
                                              0, 0);
    }
    KPROBE(3 + 4 * kb);
    uint16_t* Pw = Ps[w];
    float pds[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * (lane >> 4) + r, jj = 16 * t + (lane & 15);
        const int i = ib + r, j = j0 + jj;
        float pv = (s[t][r] > -1.0e38f) ? __expf(s[t][r] - mrow[r]) * inv[r] : 0.f;
        if (WPT)
          __builtin_amdgcn_raw_buffer_store_b16(f2bf(pv), rpt, (rowin[r] && j < T) ? (uint32_t)((prow[r] + j) * 2) : OOB,
                                                0, 0);
        float pdv = pv;
        if (drop) {   // (a zero probability stays zero either way: no per-element branch on it)
          pdv = attn_drop_keep(dkey, dpair[r], j, p.p_drop) ? pv * keep_scale : 0.f;
          pds[r] += pdv;
        }
        if (TWO_PASS && i < T && j < T) {
          const int64_t off = prow0 + (int64_t)r * p.T + j;
          if (p.P) p.P[off] = pv;
          if (p.Pd) p.Pd[off] = pdv;
        }
        Pw[ii * LDPS + jj] = f2bf(pdv);
      }
    if (drop) {
#pragma unroll
      for (int r = 0; r < 4; ++r) ps[r] += group16_sum(pds[r]);
    }
    if (!live) {
      if (!TWO_PASS) break;  // nothing to write: no P outputs in single-pass mode
      continue;              // P row tail beyond len is written as zeros; no O contribution
    }
    KPROBE(4 + 4 * kb);
    wave_lds_sync();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(Pw + (lane & 15) * LDPS + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vt + (16 * u + (lane & 15)) * LDVT + ks * 32 + 8 * (lane >> 4));
        oacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, oacc[u], 0, 0, 0);
      }
    }
    wave_lds_sync();  // Ps is rewritten by the next block
    KPROBE(5 + 4 * kb);
  }
  if (WPT && nkb < nkb_all) {   // p~ of the first key block past the valid keys: zeros
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = nkb * AKB + 16 * t + (lane & 15);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)0, rpt,
                                              (rowin[r] && j < T) ? (uint32_t)((prow[r] + j) * 2) : OOB, 0, 0);
      }
  }
  KPROBE(30);

  // ---- per-row log-sum-exp for the backward's recompute (single pass; +inf-like sentinel for rows
  // with no valid key: their P row is zero) ----
  if (!TWO_PASS && p.lse && (lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r;
      if (i < T) p.lse[bh * p.T + i] = (i < len && lrow[r] > 0.f) ? mrow[r] + logf(lrow[r]) : 3.0e38f;
    }
  }
  // ---- O -> (rows, d): the centred sum plus S_i vc ----
  float fin[4], sv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool rv_ok = ib + r < len && lrow[r] > 0.f;
    fin[r] = TWO_PASS ? 1.f : (rv_ok ? 1.f / lrow[r] : 0.f);
    sv[r] = drop ? ps[r] * fin[r] : (rv_ok ? 1.f : 0.f);
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int c = 16 * u + (lane & 15);
    const float v0 = Cn[1][c < dk ? c : 0];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r;
      if (i < T && c < dk) p.o[(b * p.T + i) * p.ldq + hoff + c] = oacc[u][r] * fin[r] + sv[r] * v0;
    }
  }
  KPROBE(31);
}

}  // namespace
}  // namespace kdfm

extern "C" int kdfm_relpos_attn_fwd(const float* qu, const float* qv, const float* qkv, const float* pos,
                                    const int64_t* lengths, float* o, float* P, float* Pdrop, float* lse,
                                    uint16_t* p_tilde, float* m_blk, int64_t B, int64_t H,
                                    int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed,
                                    uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(qu && qv && qkv && pos && o, "null pointer");
  KDFM_REQUIRE(H > 0 && d % H == 0, "d must be a multiple of H");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk <= 128 && dk % 4 == 0, "head dim must be a multiple of 4 and <= 128");
  KDFM_REQUIRE(dk <= 64 || !(P || Pdrop || p_tilde || m_blk),
               "head dims > 64: single-pass forward with lse only (the bwd2 backward's form)");
  KDFM_REQUIRE(T > 0 && T <= 4096, "T out of range");
  KDFM_REQUIRE(d % 4 == 0, "d must be a multiple of 4");
  KDFM_REQUIRE(dropout_p == 0.f || seed, "dropout needs a seed");
  KDFM_REQUIRE(!((lse || p_tilde || m_blk) && (P || Pdrop)), "lse / p~ / m_blk are single-pass outputs (no P / Pdrop)");
  KDFM_REQUIRE((p_tilde == nullptr) == (m_blk == nullptr), "p~ and m_blk go together");
  if (B == 0) return KDFM_OK;
  AttnP p;
  p.qu = qu; p.qv = qv; p.k = qkv + d; p.v = qkv + 2 * d; p.pos = pos; p.lens = lengths;
  p.o = o; p.P = P; p.Pd = Pdrop; p.lse = lse; p.pt = p_tilde; p.mblk = m_blk;
  p.B = B; p.H = H; p.T = T; p.d = d; p.dk = dk; p.ldq = d; p.ldkv = 3 * d;
  p.scale = scale; p.p_drop = dropout_p; p.seed = seed; p.rng_stream = rng_stream;
  dim3 grid((unsigned)ceil_div(T, AQ), (unsigned)(B * H));
  const bool two = P || Pdrop, wide = dk > 48;
  KDFM_REQUIRE(!p_tilde || B * H * T * T * 2 <= (int64_t)INT32_MAX, "p~ exceeds the 2 GB buffer-offset range");
  if (dk > 64)
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<false, 8>), grid, dim3(256), 0, as_stream(stream), p);
  else if (!two && p_tilde && !wide)
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<false, 3, true>), grid, dim3(256), 0, as_stream(stream), p);
  else if (!two && p_tilde)
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<false, 4, true>), grid, dim3(256), 0, as_stream(stream), p);
  else if (two && !wide)
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<true, 3>), grid, dim3(256), 0, as_stream(stream), p);
  else if (two)
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<true, 4>), grid, dim3(256), 0, as_stream(stream), p);
  else if (!wide)
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<false, 3>), grid, dim3(256), 0, as_stream(stream), p);
  else
    hipLaunchKernelGGL((relpos_attn_fwd_kernel<false, 4>), grid, dim3(256), 0, as_stream(stream), p);
  return check_launch("kdfm_relpos_attn_fwd");
}
