// Fused relative-position multi-head attention backward (bf16 MFMA 16x16x32, f32 accumulate).
//
// NeMo RelPositionMultiHeadAttention (Appendix A.7; per ConformerLayer, conformer_encoder.py:685-692):
//   S = (Qu K^T + rel_shift(Qv Ppos^T)) * scale, P = masked softmax(S), Pd = dropout(P), O = Pd V
// with rel_shift as the index map bd[i][j] = Qv_i . Ppos[T-1-i+j].  The gradients are
//   dP = dropout'(dO V^T),  r_i = sum_j dP P,  dS = P (dP - r_i) scale
//   dQu = dS K,  dQv_i = sum_j dS[i][j] Ppos[T-1-i+j],  dK = dS^T Qu,  dV = Pd^T dO,
//   dPpos[r] = sum_{b, i} dS[i][r-(T-1)+i] Qv_i.
// Nothing of size T x T is read or written: every kernel recomputes its tile of S with the
// forward's own score code (same MFMAs in the same order) and P = exp(S - lse_i) from the forward's
// per-row log-sum-exp (kdfm_relpos_attn_fwd), and r_i = sum_j dP P = dO_i . O_i (FlashAttention's
// D_i) is one row dot product over the saved forward output:
//   * kernel 1 (one workgroup per (b, h, 64 query rows), 4 waves x 16 rows): S as in the forward
//     (Qu K^T from a [key][c] K image, the positional term as G = Qv Pband^T read back skewed),
//     dPd = dO V^T, then dQu += dS K and dQv += skew(dS) Pband, the K and band operands read
//     TRANSPOSED out of the same [row][c] images with ds_read_b64_tr_b16 (one LDS image per tile);
//   * kernel 2 (one workgroup per (b, h, 64 keys), 4 waves x 16 keys): S^T = K Qu^T and the band
//     term per 16-query slice as H = Pband Qv^T (32 band rows x 16 queries) read back skewed;
//     dPd^T = V dO^T; dV += Pd^T dO and dK += dS^T Qu over all query blocks (dO / Qu read
//     transposed out of their row images);
//   * kernel 3 (one workgroup per (h, 64 relative positions, batch chunk)): dS recomputed for the
//     (i, j) diagonal band of its positions, dPpos += skew(dS)^T Qv; per-chunk partials are folded
//     in chunk order.
// The dropout mask is the forward's counter-RNG draw (same index -> same mask).  Every output
// element is owned by one workgroup and the fold is ordered: deterministic, no atomics.
#include "gemm_common.h"
#include "attn_centre.h"

// timing probe points (tools/attn_bwd_probe.hip defines KPROBE; empty in the library)
#ifndef KPROBE
#define KPROBE(i)
#endif

namespace kdfm {
namespace {

constexpr int BQ = 64;             // query rows per workgroup (kernel 1), 4 waves x 16
constexpr int BK = 64;             // keys per block
constexpr int BDK = 64;            // head dim padded to 2 MFMA k-steps
constexpr int LR = BDK + 8;        // bf16 row stride of [row][c] tiles (144 B: 8-B aligned transposed reads)
constexpr int LW = 64 + 8;         // bf16 row stride of per-wave [16][64] tiles
constexpr int PB1 = 144;           // kernel 1 band rows (127 staged; dQv's transposed reads reach row 143)
constexpr int PB = 128;            // kernel 2 / 3 band rows (127 staged)
constexpr int LG32 = 81;           // f32 stride of kernel 1's per-wave score band tile [16][80]
constexpr int LG = 96 + 8;         // bf16 row stride of the per-wave skewed dS tile [16][96]
constexpr int LH = 17;             // f32 stride of kernel 2's per-wave band tile [32][16]
constexpr int NPQ = 32;            // query rows per step of kernel 3
constexpr int NPJ = 96;            // keys per step of kernel 3 (64 positions + 31 rows of skew)
constexpr int LDL = NPJ + 8;       // bf16 row stride of kernel 3's dS tile
constexpr int LQ3 = NPQ + 8;       // bf16 row stride of kernel 3's Qv^T tile
constexpr int LG3 = 65;            // f32 stride of kernel 3's per-wave score band tile [16][64]
// per-wave scratch (bytes): kernel 1 aliases the f32 score band with the bf16 dS + skewed dS tiles,
// kernel 2 the f32 band tile with the bf16 Pd^T + dS^T tiles
constexpr int WS1 = (16 * LG32 * 4 > 16 * (LW + LG) * 2) ? 16 * LG32 * 4 : 16 * (LW + LG) * 2;
constexpr int WS2 = (32 * LH * 4 > 2 * 16 * LW * 2) ? 32 * LH * 4 : 2 * 16 * LW * 2;

struct AbP {
  const float* dO; const float* qu; const float* qv; const float* k; const float* v; const float* pos;
  const float* lse; const uint16_t* pt; const float* mblk;   // lse (B,H,T); p~ (B,H,T,T) bf16; m (B,H,T,nkb)
  const int64_t* lens;
  float* dqu; float* dqv; float* rsum; float* dk; float* dv; float* dpos_part;
  int64_t B, H, T, d, dkh, ldq, ldkv;
  float scale, p_drop;
  const uint64_t* seed; uint64_t rng_stream;
  int bpc;   // batches per chunk (kernel 3)
  // bwd2: dS and Pd (dropout-applied P) as bf16 (B, H, T, ldt), written by kernel 1, read by kernels 2b / 3b
  uint16_t* ds; uint16_t* pdo; int64_t ldt;
  const float* O;   // bwd2: the forward output (row sums formed in the dQ kernel)
  // bwd2 over prepared operands (csrc/attn_fwd3.hip): bf16 centred K / V tiles (B*H, Tp, LR), the centre
  // (B*H, 2, DKP), this layer's band rows (H, npb, LR)
  const uint16_t* kb; const uint16_t* vb; const float* cen; const uint16_t* pb; int64_t Tp, npb;
};

constexpr uint32_t AB_OOB = 0x80000000u;   // buffer offset past every buffer: the access is dropped / reads 0

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

// columns c0 .. c0 + 7 of a row (head = the row's first column of this head) as bf16, zero past `valid`;
// both loads unconditional (column clamped) and masked by a multiply: a conditional load, or a select
// on a loaded value, is branched around and waited for one at a time
__device__ __forceinline__ bf16x8 frag8(const float* head, int c0, int valid) {
  const float m0 = valid >= 4 ? 1.f : 0.f, m1 = valid >= 8 ? 1.f : 0.f;
  const float4 a = *reinterpret_cast<const float4*>(head + (valid >= 4 ? c0 : 0));
  const float4 b = *reinterpret_cast<const float4*>(head + (valid >= 8 ? c0 + 4 : 0));
  const float t[8] = {a.x * m0, a.y * m0, a.z * m0, a.w * m0, b.x * m1, b.y * m1, b.z * m1, b.w * m1};
  return pack_bf16x8<bf16x8>(t);
}

typedef short bf16x4 __attribute__((ext_vector_type(4)));
// 4 consecutive bf16 of a row (the 16-wide tail k-step over a head dim padded to 48); columns at or past
// `valid` read as 0
__device__ __forceinline__ bf16x4 frag4(const float* head, int c0, int valid) {
  const float m = valid >= 4 ? 1.f : 0.f;
  const float4 a = *reinterpret_cast<const float4*>(head + (valid >= 4 ? c0 : 0));
  return __builtin_bit_cast(bf16x4, make_uint2(pack_bf16x2(a.x * m, a.y * m), pack_bf16x2(a.z * m, a.w * m)));
}

// MFMA 16x16x32 operand read TRANSPOSED out of a [k][n] bf16 LDS image (row stride ld elements):
// lane l receives X[k0 + 8*(l>>4) + e][n0 + (l & 15)], e = 0..7 -- the B operand X[k][n], or the A
// operand of X^T.  Two ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q, columns
// 4p..4p+3 of a 4-row block and receives column (l & 15) of the block's 4 rows.  EXEC must be full.
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* img, int ld, int k0, int n0, int lane) {
  const int li = lane & 15;
  const uint16_t* a = img + (k0 + 8 * (lane >> 4) + (li >> 2)) * ld + n0 + 4 * (li & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a + 4 * ld));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
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
template <int MAXI, int LDR = LR>
__device__ __forceinline__ void put_rows(uint16_t* rc, uint16_t* cr, int ldt, const float4 (&v)[MAXI], int n, int dk) {
  const int cq = dk >> 2;
#pragma unroll
  for (int it = 0; it < MAXI; ++it) {
    const int e = threadIdx.x + it * 256;
    if (e >= n * cq) continue;
    const int rr = e / cq, c4 = (e - rr * cq) * 4;
    if (rc) st4(rc + rr * LDR + c4, v[it]);
    if (cr) {
      cr[(c4 + 0) * ldt + rr] = f2bf(v[it].x);
      cr[(c4 + 1) * ldt + rr] = f2bf(v[it].y);
      cr[(c4 + 2) * ldt + rr] = f2bf(v[it].z);
      cr[(c4 + 3) * ldt + rr] = f2bf(v[it].w);
    }
  }
}

// fetch_rows as buffer loads: an out-of-range row's offset is AB_OOB (the load reads 0 without a memory
// access), so no load is branched around and no 64-bit address is held per load; `rsrc` covers `src`
template <int MAXI>
__device__ __forceinline__ void fetch_rows_b(float4 (&v)[MAXI], __amdgpu_buffer_rsrc_t rsrc, int64_t ld,
                                             int64_t base_row, int r0, int n, int lo, int hi, int64_t c0, int dk) {
  const int cq = dk >> 2;
#pragma unroll
  for (int it = 0; it < MAXI; ++it) {
    const int e = threadIdx.x + it * 256;
    const int rr = e / cq, c4 = (e - rr * cq) * 4;
    const int r = r0 + rr;
    const bool ok = e < n * cq && r >= lo && r < hi;
    const uint32_t off = ok ? (uint32_t)(((base_row + r) * ld + c0 + c4) * 4) : 0x80000000u;
    v[it] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
  }
}

// zero columns [dk, 64) of rows [0, rows) of a [row][c] image, and every column of rows [z0, rows)
__device__ __forceinline__ void zero_pad(uint16_t* img, int rows, int dk, int z0) {
  for (int e = threadIdx.x; e < rows * (BDK - dk); e += 256) img[(e / (BDK - dk)) * LR + dk + e % (BDK - dk)] = 0;
  for (int e = threadIdx.x; e < (rows - z0) * dk; e += 256) img[(z0 + e / dk) * LR + e % dk] = 0;
}

// zero a whole [rows][LR] image with 16-byte stores (the bwd2 kernels: a superset of zero_pad -- the data
// columns of rows below z0 are rewritten by put_rows after a barrier -- without its per-element divisions)
template <int LDR = LR>
__device__ __forceinline__ void zero_img(uint16_t* img, int rows) {
  static_assert((LDR * 2) % 16 == 0, "row stride must be a multiple of 16 bytes");
  for (int e = threadIdx.x; e < rows * LDR / 8; e += 256) reinterpret_cast<uint4*>(img)[e] = make_uint4(0u, 0u, 0u, 0u);
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
// RIN: the row sums r_i are formed in the prologue from dO and O (p.O) instead of read from p.rsum
// NU = 8 (head dim <= 128, FastConformer-XL): the head dim is padded to 4 MFMA k-steps (KS) instead of 2.
// PREP (bwd2 only): K / V / band tiles copied by LDS-DMA from the forward's prepared bf16 operands
// (kdfm_attn_kv_prep / kdfm_attn_band_prep, the same bf16(K - kc) / bf16(V - vc) values the register path
// stages) and the centre read from them -- no staging registers, no conversion or centring pass
template <int NU, bool SAVE = false, bool RIN = false, bool PREP = false>
__global__ __launch_bounds__(256, NU == 3 ? 2 : 1) void attn_bwd_dq_kernel(AbP p) {
  // the prepared tiles (PREP) pad head dims <= 48 to 48 (attn_prep_dkp): one 32-wide and one 16-wide MFMA
  // k-step over the head dim; the register-staged forms pad to 64 / 128
  constexpr int DKP = (PREP && NU == 3) ? 48 : 32 * (NU > 4 ? 4 : 2);
  constexpr int KS = DKP / 32;
  constexpr bool TAIL = DKP % 32 != 0;
  constexpr int LRK = DKP + 8;
  static_assert(SAVE || KS == 2, "the pre-bwd2 path covers head dims <= 64 only");
  static_assert(!PREP || (SAVE && RIN), "prepared operands: the bwd2 dQ kernel only");
  constexpr int KCH = BK * LRK * 2 / 1024;                  // 1 KB DMA chunks of a K / V tile
  constexpr int PCH = (PB1 * LRK * 2 + 1023) / 1024;        // ... of the band (rows past 143 unused)
  static_assert(BK * LRK * 2 % 1024 == 0, "K / V tiles must be whole 1 KB chunks");
  __shared__ __attribute__((aligned(16))) uint16_t Ks[BK * LRK];     // K block [key][c]
  __shared__ __attribute__((aligned(16))) uint16_t Vs[BK * LRK];     // V block [key][c]
  __shared__ __attribute__((aligned(16))) uint16_t Pr[PREP ? PCH * 512 : PB1 * LRK];    // Ppos band [band row][c]
  __shared__ __attribute__((aligned(16))) float Wsc[4][WS1 / 4];    // per-wave scratch
  // SAVE (bwd2): per wave dS^T and Pd^T tiles [64 keys][16 rows] bf16 (4 rows of a key per 8-byte write); dS and
  // Pd leave as 16-byte buffer stores of transposed reads (fixed count per lane and key block, out-of-range
  // chunks dropped by the range check), the dS read doubling as dQu's A fragment
  __shared__ __attribute__((aligned(16))) uint16_t Tw[SAVE ? 4 : 1][SAVE ? 2 * BK * 16 : 8];
  __shared__ __attribute__((aligned(16))) float Cn[2][DKP];   // the forward's key / value centre (attn_centre.h)

  KPROBE(0);
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
  if constexpr (PREP) {
    // (the DMA'd tiles are complete images: padding columns / rows come zero from the preparation)
  } else if constexpr (SAVE) {
    zero_img<LRK>(Ks, BK);
    zero_img<LRK>(Vs, BK);
    zero_img<LRK>(Pr, PB1);
  } else {
    zero_pad(Ks, BK, dk, BK);
    zero_pad(Vs, BK, dk, BK);
    zero_pad(Pr, PB1, dk, 127);
  }

  // this lane's query row (A-fragment row): Qu, Qv and dO fragments
  const int iq = i0 + w * 16 + (lane & 15);
  bf16x8 fu[KS], fv[KS], fdo[KS];
  bf16x4 fut = {}, fvt = {}, fdot = {};   // TAIL: columns 32 KS + 4 (lane >> 4) .. + 3
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int c0 = ks * 32 + 8 * (lane >> 4);
    const int valid = iq < T ? dk - c0 : 0;
    const int64_t off = (b * p.T + (iq < T ? iq : 0)) * p.ldq + hoff;
    fu[ks] = frag8(p.qu + off, c0, valid);
    fv[ks] = frag8(p.qv + off, c0, valid);
    fdo[ks] = frag8(p.dO + off, c0, valid);
  }
  if constexpr (TAIL) {
    const int c0 = KS * 32 + 4 * (lane >> 4);
    const int valid = iq < T ? dk - c0 : 0;
    const int64_t off = (b * p.T + (iq < T ? iq : 0)) * p.ldq + hoff;
    fut = frag4(p.qu + off, c0, valid);
    fvt = frag4(p.qv + off, c0, valid);
    fdot = frag4(p.dO + off, c0, valid);
  }
  const int ib = i0 + w * 16 + 4 * (lane >> 4);   // C-layout rows ib + r
  const int64_t prow0 = (bh * p.T + ib) * p.T;
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const float keep = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  // r_i = sum_j dP P = dO_i . O_i (attn_rowdot_kernel, before this kernel) and the forward's lse_i
  float rs[4], ls[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool ok = ib + r < len;
    rs[r] = (ok && !RIN) ? p.rsum[bh * p.T + ib + r] : 0.f;
    ls[r] = ok ? p.lse[bh * p.T + ib + r] : 3.0e38f;
  }

  // bwd2 (SAVE): the forward's softmax in the exp2 domain (P = exp2(s_raw scale log2e - lse log2e)), S_bd by lane
  // permutes of the G accumulators (attn_fwd3.hip: S_bd(t, r) = G[t + (off >= 16)][r] of lane (off & 15) + 16 q4),
  // and the dropout pair hashes shared between neighbouring lanes (common.h attn_drop_keep: keys 16 t + lo and
  // 16 t + (lo ^ 1) share one; even lanes hash rows ib, ib + 1, odd lanes ib + 2, ib + 3)
  const int q4 = lane >> 4, lo = lane & 15;
  const bool odd = lo & 1;
  const float sl2 = p.scale * 1.4426950408889634f;
  float ls2[4];
  int bsrc_lane[4];
  bool bhi[4];
  uint64_t dpr[2];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ls2[r] = ls[r] * 1.4426950408889634f;
    const int off = lo - 4 * q4 - r + 15;   // 0 .. 30
    bsrc_lane[r] = ((off & 15) + 16 * q4) * 4;
    bhi[r] = off >= 16;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) dpr[k] = attn_drop_rowpairs(bh * p.T + ib + (odd ? 2 : 0) + k, p.T) + (uint64_t)(lo >> 1);
  const uint64_t dkey = rng_key(seed, p.rng_stream);
  const uint32_t thr = drop_threshold(p.p_drop);
  const int hsh = odd ? 16 : 0;

  // next key block's operands in registers: V and K rows, the Ppos band
  float4 nv[NU], nk[NU], nb[2 * NU];
  // bwd2 (SAVE): buffer loads over K / V (qkv rows) and the band (the entry checks the sizes fit 31 bits)
  const int kvbytes = SAVE ? (int)((p.B * p.T * p.ldkv - p.d) * 4) : 0;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)p.k, (short)0, kvbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)p.v, (short)0, kvbytes - (int)(4 * p.d) * SAVE,
                                                                      0x00020000);
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)p.pos, (short)0,
                                                                      SAVE ? (int)(npos * p.d * 4) : 0, 0x00020000);
  auto fetch = [&](int kb) {
    const int j0 = kb * BK;
    const int rbase = T - 1 - (i0 + BQ - 1) + j0;
    if constexpr (PREP) {
      typedef __attribute__((address_space(3))) void lds_t;
      typedef __attribute__((address_space(1))) void gl_t;
      const uint4* ks = reinterpret_cast<const uint4*>(p.kb + (bh * p.Tp + j0) * LRK);
      const uint4* vs = reinterpret_cast<const uint4*>(p.vb + (bh * p.Tp + j0) * LRK);
      const uint4* bs = reinterpret_cast<const uint4*>(p.pb + (h * p.npb + rbase + 64) * LRK);
#pragma unroll
      for (int i = 0; i < (2 * KCH + PCH + 3) / 4; ++i) {
        const int f = w + 4 * i;   // wave-uniform
        if (f < KCH)
          __builtin_amdgcn_global_load_lds((gl_t*)(ks + f * 64 + lane), (lds_t*)(reinterpret_cast<uint4*>(Ks) + f * 64),
                                           16, 0, 0);
        else if (f < 2 * KCH)
          __builtin_amdgcn_global_load_lds((gl_t*)(vs + (f - KCH) * 64 + lane),
                                           (lds_t*)(reinterpret_cast<uint4*>(Vs) + (f - KCH) * 64), 16, 0, 0);
        else if (f < 2 * KCH + PCH)
          __builtin_amdgcn_global_load_lds((gl_t*)(bs + (f - 2 * KCH) * 64 + lane),
                                           (lds_t*)(reinterpret_cast<uint4*>(Pr) + (f - 2 * KCH) * 64), 16, 0, 0);
      }
    } else if constexpr (SAVE) {
      fetch_rows_b<NU>(nv, rv, p.ldkv, b * p.T, j0, BK, 0, len, hoff, dk);
      fetch_rows_b<NU>(nk, rk, p.ldkv, b * p.T, j0, BK, 0, len, hoff, dk);
      fetch_rows_b<2 * NU>(nb, rp, p.d, 0, rbase, 127, 0, npos, hoff, dk);
    } else {
      fetch_rows<NU>(nv, p.v, p.ldkv, b * p.T, j0, BK, 0, len, hoff, dk);
      fetch_rows<NU>(nk, p.k, p.ldkv, b * p.T, j0, BK, 0, len, hoff, dk);
      fetch_rows<2 * NU>(nb, p.pos, p.d, 0, rbase, 127, 0, npos, hoff, dk);
    }
  };
  if constexpr (SAVE) {   // the first block's loads in flight behind the centre and row-sum prologue
    if (nkb > 0) fetch(0);
  }

  // the forward's centring (attn_centre.h): K rows staged as K_j - kc (the scores, hence P = exp(s - lse),
  // are the forward's), V rows as V_j - vc with cs_i = dO_i . vc added back to dPd in f32
  if constexpr (PREP) {
    for (int e = threadIdx.x; e < 2 * DKP; e += 256) Cn[e / DKP][e % DKP] = p.cen[bh * 2 * DKP + e];
    __syncthreads();
  } else {
    kv_centre<DKP>(p.k + b * p.T * p.ldkv + hoff, p.v + b * p.T * p.ldkv + hoff, p.ldkv, len, dk, Cn);
  }
  // cs_i for this lane's C-layout rows: row (lane & 15) of the wave's 16 dotted in f32 by its 4 lane groups
  // (16 columns each), summed across them, then picked up by the lanes owning each row.  With RIN (bwd2)
  // the row sums r_i = dO_i . O_i are formed the same way here instead of by attn_rowdot_kernel
  float cs[4], rin[4];
  {
    const int q = lane >> 4;
    float part = 0.f, pr = 0.f;
    if (iq < T) {
      const float* dor = p.dO + (b * p.T + iq) * p.ldq + hoff;
      const float* orow = p.O + (b * p.T + iq) * p.ldq + hoff;
#pragma unroll
      for (int c4 = 0; c4 < DKP / 16; ++c4) {
        const int c = (DKP / 4) * q + 4 * c4;
        if (c < dk) {
          const float4 g = *reinterpret_cast<const float4*>(dor + c);
          part += g.x * Cn[1][c] + g.y * Cn[1][c + 1] + g.z * Cn[1][c + 2] + g.w * Cn[1][c + 3];
          if (RIN) {
            const float4 o = *reinterpret_cast<const float4*>(orow + c);
            pr += g.x * o.x + g.y * o.y + g.z * o.z + g.w * o.w;
          }
        }
      }
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    if (RIN) {
      pr += __shfl_xor(pr, 16, 64);
      pr += __shfl_xor(pr, 32, 64);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cs[r] = __shfl(part, 4 * q + r, 64);
      rin[r] = RIN ? __shfl(pr, 4 * q + r, 64) : 0.f;
    }
  }
  if (RIN) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rs[r] = ib + r < len ? rin[r] : 0.f;
  }
  // subtract the centre (read back from LDS: holding it in registers spills the loop's staging addresses)
  // from the staged rows of keys [j0, j0 + BK) that are valid (rows past len stay 0)
  auto centre = [&](float4 (&v)[NU], const float* c, int j0) {
    const int cq = dk >> 2;
#pragma unroll
    for (int it = 0; it < NU; ++it) {
      const int e = threadIdx.x + it * 256;
      const int rr = e / cq;
      const float m = (e < BK * cq && j0 + rr < len) ? 1.f : 0.f;   // a multiply: no branch around the read
      const float4 cc = *reinterpret_cast<const float4*>(c + (e - rr * cq) * 4);
      v[it] = make_float4(v[it].x - m * cc.x, v[it].y - m * cc.y, v[it].z - m * cc.z, v[it].w - m * cc.w);
    }
  };

  f32x4 aq[NU], av[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) { aq[u] = f32x4{0.f, 0.f, 0.f, 0.f}; av[u] = aq[u]; }
  const int wb = 48 - 16 * w;   // this wave's band offset
  float* G = Wsc[w];                                    // f32 score band [16][LG32]
  uint16_t* D = reinterpret_cast<uint16_t*>(Wsc[w]);    // bf16 dS [16][LW]   (after the scores)
  uint16_t* Gk = D + 16 * LW;                           // bf16 skewed dS [16][LG]
  const int sbytes = SAVE ? (int)(p.B * p.H * p.T * p.ldt * 2) : 0;
  const __amdgpu_buffer_rsrc_t rds = __builtin_amdgcn_make_buffer_rsrc((void*)p.ds, (short)0, sbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rpd = __builtin_amdgcn_make_buffer_rsrc((void*)p.pdo, (short)0, sbytes, 0x00020000);
  if (!SAVE && nkb > 0) fetch(0);
  KPROBE(1);
  for (int kb = 0; kb < nkb; ++kb) {
    const int j0 = kb * BK;
    if constexpr (PREP) {
      if (kb > 0) {
        __syncthreads();   // every wave is done with the previous block's tiles
        fetch(kb);
      }
      __builtin_amdgcn_s_waitcnt(0x70);   // vmcnt(0) lgkmcnt(0): this wave's DMA chunks (and its stores) landed
      __syncthreads();
    } else {
      __syncthreads();
      centre(nk, Cn[0], j0);
      centre(nv, Cn[1], j0);
      put_rows<NU, LRK>(Vs, nullptr, 0, nv, BK, dk);
      put_rows<NU, LRK>(Ks, nullptr, 0, nk, BK, dk);
      put_rows<2 * NU, LRK>(Pr, nullptr, 0, nb, 127, dk);
      __syncthreads();
      if (kb + 1 < nkb) fetch(kb + 1);
    }
    KPROBE(2 + 4 * kb);
    // ---- S of this wave's 16 rows x 64 keys: the forward's scores (relpos_attn_fwd_kernel) ----
    float s[4][4];
    {
      f32x4 ac[4], g[5];
#pragma unroll
      for (int t = 0; t < 4; ++t) ac[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 5; ++t) g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int kof = ks * 32 + 8 * (lane >> 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 kbf = *reinterpret_cast<const bf16x8*>(Ks + (16 * t + (lane & 15)) * LRK + kof);
          ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fu[ks], kbf, ac[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const bf16x8 pb = *reinterpret_cast<const bf16x8*>(Pr + (wb + 16 * t + (lane & 15)) * LRK + kof);
          g[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fv[ks], pb, g[t], 0, 0, 0);
        }
      }
      if constexpr (TAIL) {
        const int kof = KS * 32 + 4 * (lane >> 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x4 kbf = *reinterpret_cast<const bf16x4*>(Ks + (16 * t + (lane & 15)) * LRK + kof);
          ac[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fut, kbf, ac[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const bf16x4 pb = *reinterpret_cast<const bf16x4*>(Pr + (wb + 16 * t + (lane & 15)) * LRK + kof);
          g[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fvt, pb, g[t], 0, 0, 0);
        }
      }
      if constexpr (SAVE) {   // raw scores ac + bd (the validity select and the scale come with the exp2 below)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float X[5];
#pragma unroll
          for (int t = 0; t < 5; ++t) {
            const float gv = g[t][r];   // (copied out: a bit_cast of the vector element read element 0)
            X[t] = __int_as_float(__builtin_amdgcn_ds_bpermute(bsrc_lane[r], __float_as_int(gv)));
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) s[t][r] = ac[t][r] + (bhi[r] ? X[t + 1] : X[t]);
        }
      } else {
#pragma unroll
        for (int t = 0; t < 5; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) G[(4 * (lane >> 4) + r) * LG32 + 16 * t + (lane & 15)] = g[t][r];
        wsync();
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ii = 4 * (lane >> 4) + r, jj = 16 * t + (lane & 15);
            const float bd = G[ii * LG32 + jj - ii + 15];
            s[t][r] = (j0 + jj < len) ? (ac[t][r] + bd) * p.scale : -3.0e38f;
          }
        wsync();   // the scratch is rewritten below
      }
    }
    KPROBE(3 + 4 * kb);
    // ---- dPd = dO V^T ----
    f32x4 a[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vs + (16 * t + (lane & 15)) * LRK + ks * 32 + 8 * (lane >> 4));
        a[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fdo[ks], vb, a[t], 0, 0, 0);
      }
    if constexpr (TAIL) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x4 vb = *reinterpret_cast<const bf16x4*>(Vs + (16 * t + (lane & 15)) * LRK + KS * 32 + 4 * (lane >> 4));
        a[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fdot, vb, a[t], 0, 0, 0);
      }
    }
    for (int e = lane; e < 16 * LG / 2; e += 64) reinterpret_cast<uint32_t*>(Gk)[e] = 0u;
    bf16x8 dfr[2];   // dQu's A fragments (rows lane & 15, keys ks 32 + 8 q4 ..)
    if constexpr (SAVE) {
      uint16_t* Dt = Tw[w];             // dS^T [key][16 rows]
      uint16_t* Pt = Tw[w] + BK * 16;   // Pd^T
      uint32_t hk[4][2], hp[4][2];
      if (p.p_drop > 0.f) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int k = 0; k < 2; ++k) hk[t][k] = drop_pair_bits(dkey, dpr[k] + (uint64_t)((j0 >> 1) + 8 * t));
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int k = 0; k < 2; ++k) hp[t][k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hk[t][k], 0xB1, 0xF, 0xF, false);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = j0 + 16 * t + lo;
        float dsv[4], pdv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = ib + r < len && j < len;
          float g = a[t][r] + cs[r];
          bool kp = true;
          if (p.p_drop > 0.f) {
            const uint32_t hv = ((r >> 1) == (int)odd) ? hk[t][r & 1] : hp[t][r & 1];
            kp = ((hv >> hsh) & 0xffffu) >= thr;
            g = kp ? g * keep : 0.f;
          }
          const float pe = __builtin_amdgcn_exp2f(__builtin_fmaf(s[t][r], sl2, -ls2[r]));
          dsv[r] = ok ? pe * (g - rs[r]) * p.scale : 0.f;
          pdv[r] = (ok && kp) ? pe * keep : 0.f;
          const int ii = 4 * q4 + r, jj = 16 * t + lo;
          Gk[ii * LG + jj - ii + 15] = f2bf(dsv[r]);
        }
        *reinterpret_cast<uint2*>(Dt + (16 * t + lo) * 16 + 4 * q4) =
            make_uint2(pack_bf16x2(dsv[0], dsv[1]), pack_bf16x2(dsv[2], dsv[3]));
        *reinterpret_cast<uint2*>(Pt + (16 * t + lo) * 16 + 4 * q4) =
            make_uint2(pack_bf16x2(pdv[0], pdv[1]), pack_bf16x2(pdv[2], pdv[3]));
      }
      wsync();
      // this wave's 16 rows x 64 keys of dS and Pd: lane (q4, lo) stores row lo's keys ks 32 + 8 q4 .. + 7 (a
      // transposed read of the [key][row] tile), two chunks per lane each
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int i = i0 + w * 16 + lo, jc = j0 + ks * 32 + 8 * q4;
        const uint32_t off = (i < T && jc < p.ldt) ? (uint32_t)(((bh * p.T + i) * p.ldt + jc) * 2) : AB_OOB;
        dfr[ks] = tr_frag(Dt, 16, ks * 32, 0, lane);
        const bf16x8 vp = tr_frag(Pt, 16, ks * 32, 0, lane);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, dfr[ks]),
                                               rds, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, vp), rpd,
                                               off, 0, 0);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = ib + r, j = j0 + 16 * t + (lane & 15);
          float ds = 0.f;
          if (i < len && j < len) {
            float g = a[t][r] + cs[r];
            if (p.p_drop > 0.f) {
              const bool kp = attn_drop_keep(dkey, attn_drop_rowpairs(bh * p.T + i, p.T), j, p.p_drop);
              g = kp ? g * keep : 0.f;
            }
            const float pe = __expf(s[t][r] - ls[r]);
            ds = pe * (g - rs[r]) * p.scale;
          }
          const int ii = 4 * (lane >> 4) + r, jj = 16 * t + (lane & 15);
          const uint16_t bv = f2bf(ds);
          D[ii * LW + jj] = bv;
          Gk[ii * LG + jj - ii + 15] = bv;
        }
      wsync();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        dfr[ks] = *reinterpret_cast<const bf16x8*>(D + (lane & 15) * LW + ks * 32 + 8 * (lane >> 4));
    }
    KPROBE(4 + 4 * kb);
    // ---- dQu += dS K (K read transposed), dQv += skew(dS) Pband (band read transposed) ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int u = 0; u < NU; ++u) aq[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dfr[ks], tr_frag(Ks, LRK, ks * 32, 16 * u, lane),
                                                                                aq[u], 0, 0, 0);
    }
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const bf16x8 ga = *reinterpret_cast<const bf16x8*>(Gk + (lane & 15) * LG + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int u = 0; u < NU; ++u)
        av[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, tr_frag(Pr, LRK, wb + ks * 32, 16 * u, lane), av[u], 0, 0, 0);
    }
    wsync();
    KPROBE(5 + 4 * kb);
  }
  KPROBE(30);
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r, c = 16 * u + (lane & 15);
      if (i < T && c < dk) {
        const int64_t off = (b * p.T + i) * p.ldq + hoff + c;
        p.dqu[off] = aq[u][r];
        p.dqv[off] = av[u][r];
      }
    }
  KPROBE(31);
}

// ---------------------------------------------------------------------------------------------
// kernel 2: dK, dV  (P = p~ exp(m_ikb - lse_i) read from the forward's bf16 p~ and block maxima)
// ---------------------------------------------------------------------------------------------
template <int NU>
__global__ __launch_bounds__(256, NU == 3 ? 2 : 1) void attn_bwd_dkv_kernel(AbP p) {
  __shared__ __attribute__((aligned(16))) uint16_t Os[BQ * LR];     // dO block [query][c]
  __shared__ __attribute__((aligned(16))) uint16_t Qs[BQ * LR];     // Qu block [query][c]
  __shared__ __attribute__((aligned(16))) float Pt[BK * (BQ + 1)];  // P block^T [key][query]
  __shared__ __attribute__((aligned(16))) uint16_t Pw[4][16 * LW];  // per wave Pd^T [key][query]
  __shared__ __attribute__((aligned(16))) uint16_t Dw[4][16 * LW];  // per wave dS^T [key][query]
  __shared__ float Rs[BQ], Cs[BQ];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const Blk3 blk = xcd_block3();
  const int64_t bh = blk.y;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int j0 = (int)blk.x * BK;   // = kb * 64: this workgroup's keys lie in one block of the forward
  const int kb = (int)blk.x;
  const int nkb_all = (T + BK - 1) / BK;
  const int len = p.lens ? (int)min<int64_t>(p.lens[b], p.T) : T;
  const int64_t hoff = h * p.dkh;
  zero_pad(Os, BQ, dk, BQ);
  zero_pad(Qs, BQ, dk, BQ);

  const int jk = j0 + w * 16 + (lane & 15);   // A-fragment row (key)
  bf16x8 fv[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c0 = ks * 32 + 8 * (lane >> 4);
    const bool ok = jk < len;
    fv[ks] = frag8(p.v + (b * p.T + (ok ? jk : 0)) * p.ldkv + hoff, c0, ok ? dk - c0 : 0);
  }
  const int jb = j0 + w * 16 + 4 * (lane >> 4);   // C-layout key rows jb + r
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const float keep = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  f32x4 adv[NU], adk[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) { adv[u] = f32x4{0.f, 0.f, 0.f, 0.f}; adk[u] = adv[u]; }
  uint16_t* PW = Pw[w];
  uint16_t* DW = Dw[w];
  const int nqb = (j0 < len) ? (len + BQ - 1) / BQ : 0;   // query rows >= len have P == 0
  // next query block's operands in registers: dO and Qu rows, the p~ block (row-major, coalesced along
  // keys), the row sums and the rows' scales exp(m_ikb - lse_i)
  float4 ndo[NU], nqu[NU];
  uint16_t npb[BQ * BK / 256];
  float nrs = 0.f, nm = 0.f, nl = 3.0e38f;
  auto fetch = [&](int qb) {
    const int i0 = qb * BQ;
    fetch_rows<NU>(ndo, p.dO, p.ldq, b * p.T, i0, BQ, 0, T, hoff, dk);
    fetch_rows<NU>(nqu, p.qu, p.ldq, b * p.T, i0, BQ, 0, T, hoff, dk);
#pragma unroll
    for (int it = 0; it < BQ * BK / 256; ++it) {
      const int e = threadIdx.x + it * 256;
      const int ii = e / BK, kk = e - ii * BK;
      const int i = i0 + ii, j = j0 + kk;
      npb[it] = (i < len && j < len) ? p.pt[(bh * p.T + i) * p.T + j] : (uint16_t)0;
    }
    if (threadIdx.x < BQ) {
      const int i = i0 + (int)threadIdx.x;
      const bool ok = i < len;
      nrs = ok ? p.rsum[bh * p.T + i] : 0.f;
      nm = ok ? p.mblk[(bh * p.T + i) * nkb_all + kb] : 0.f;
      nl = ok ? p.lse[bh * p.T + i] : 3.0e38f;
    }
  };
  if (nqb > 0) fetch(0);
  for (int qb = 0; qb < nqb; ++qb) {
    const int i0 = qb * BQ;
    __syncthreads();
    put_rows<NU>(Os, nullptr, 0, ndo, BQ, dk);
    put_rows<NU>(Qs, nullptr, 0, nqu, BQ, dk);
#pragma unroll
    for (int it = 0; it < BQ * BK / 256; ++it) {
      const int e = threadIdx.x + it * 256;
      const int ii = e / BK, kk = e - ii * BK;
      Pt[kk * (BQ + 1) + ii] = __uint_as_float((uint32_t)npb[it] << 16);
    }
    if (threadIdx.x < BQ) {
      Rs[threadIdx.x] = nrs;
      Cs[threadIdx.x] = __expf(nm - nl);
    }
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
        if (j < len && i < len) {
          const float pv = Pt[(j - j0) * (BQ + 1) + qq] * Cs[qq];
          float g = a[t][r];
          pd = pv;
          if (p.p_drop > 0.f) {
            const bool kp = attn_drop_keep(rng_key(seed, p.rng_stream), attn_drop_rowpairs(bh * p.T + i, p.T), j, p.p_drop);
            g = kp ? g * keep : 0.f;
            pd = kp ? pv * keep : 0.f;
          }
          ds = pv * (g - Rs[qq]) * p.scale;
        }
        PW[kk * LW + qq] = f2bf(pd);
        DW[kk * LW + qq] = f2bf(ds);
      }
    wsync();
    // dV += Pd^T dO, dK += dS^T Qu (dO / Qu read transposed out of their row images)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(PW + (lane & 15) * LW + ks * 32 + 8 * (lane >> 4));
      const bf16x8 da = *reinterpret_cast<const bf16x8*>(DW + (lane & 15) * LW + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        adv[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, tr_frag(Os, LR, ks * 32, 16 * u, lane), adv[u], 0, 0, 0);
        adk[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, tr_frag(Qs, LR, ks * 32, 16 * u, lane), adk[u], 0, 0, 0);
      }
    }
    wsync();
  }
#pragma unroll
  for (int u = 0; u < NU; ++u)
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
// kernel 3: per-chunk partials of dPpos  (P from p~ and the block maxima, as kernel 2)
// ---------------------------------------------------------------------------------------------
template <int NU>
__global__ __launch_bounds__(256, NU == 3 ? 2 : 1) void attn_bwd_dpos_kernel(AbP p) {
  __shared__ __attribute__((aligned(16))) uint16_t Vs[NPJ * LR];     // V rows jbase.. [key][c]
  __shared__ __attribute__((aligned(16))) uint16_t Dl[NPQ * LDL];    // dS [i - ib0][j - jbase]
  __shared__ __attribute__((aligned(16))) uint16_t Qt[BDK * LQ3];    // Qv^T [c][i - ib0]
  __shared__ float Rs[NPQ];
  __shared__ float Cs[NPQ * 3];   // exp(m_{i,kb} - lse_i) of the (up to) 3 key blocks the 96 keys touch

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const int npos = 2 * T - 1;
  const int nkb_all = (T + BK - 1) / BK;
  const Blk3 blk = xcd_block3();
  const int r0 = (int)blk.x * 64;
  const int64_t h = blk.y;
  const int64_t bchunk = blk.z;
  const int64_t hoff = h * p.dkh;
  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const float keep = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  zero_pad(Vs, NPJ, dk, NPJ);
  for (int e = threadIdx.x; e < (BDK - dk) * LQ3; e += 256) Qt[dk * LQ3 + e] = 0;
  f32x4 acc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
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
  // next iteration's operands in registers (software pipeline): V rows, Qv rows, row sums, the rows'
  // block scales, this lane's dO fragments and 12 p~ elements
  float4 nvr[(NPJ * 4 * NU + 255) / 256], nqr[(NPQ * 4 * NU + 255) / 256];
  float nrs = 0.f, nm = 0.f, nl = 3.0e38f;
  bf16x8 nfdo[2];
  uint16_t np[3][4];
  auto kbase = [&](int jb) { return (jb > 0 ? jb : 0) >> 6; };
  auto fetch = [&](int64_t bb, int ib, int ln) {
    const int jb = r0 - (T - 1) + ib;
    const int64_t bhh = bb * p.H + h;
    fetch_rows<(NPJ * 4 * NU + 255) / 256>(nvr, p.v, p.ldkv, bb * p.T, jb, NPJ, 0, ln, hoff, dk);
    fetch_rows<(NPQ * 4 * NU + 255) / 256>(nqr, p.qv, p.ldq, bb * p.T, ib, NPQ, 0, ln, hoff, dk);
    if (threadIdx.x < NPQ) nrs = (ib + (int)threadIdx.x < ln) ? p.rsum[bhh * p.T + ib + threadIdx.x] : 0.f;
    if (threadIdx.x < 3 * NPQ) {
      const int il = threadIdx.x / 3, q = threadIdx.x - 3 * il;
      const int i = ib + il, kb = kbase(jb) + q;
      const bool ok = i < ln && kb < nkb_all;
      nm = ok ? p.mblk[(bhh * p.T + i) * nkb_all + kb] : 0.f;
      nl = ok ? p.lse[bhh * p.T + i] : 3.0e38f;
    }
    const int iq = ib + 16 * qh + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c0 = ks * 32 + 8 * (lane >> 4);
      const bool ok = iq < ln;
      nfdo[ks] = frag8(p.dO + (bb * p.T + (ok ? iq : 0)) * p.ldq + hoff, c0, ok ? dk - c0 : 0);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 16 * qh + 4 * (lane >> 4) + r, jl = 48 * kh + 16 * t + (lane & 15);
        const int i = ib + il, j = jb + jl;
        np[t][r] = (i < ln && j >= 0 && j < ln) ? p.pt[(bhh * p.T + i) * p.T + j] : (uint16_t)0;
      }
  };
  int64_t b = b0;
  int ib0 = -NPQ, len = b0 < b1 ? ulen(b0) : 0;
  bool more = b0 < b1 && advance(b, ib0, len);
  if (more) fetch(b, ib0, len);
  while (more) {
    const int64_t bh = b * p.H + h;
    const int jbase = r0 - (T - 1) + ib0;
    const int kb0 = kbase(jbase);
    const int cur_len = len;
    const int cur_ib0 = ib0;
    __syncthreads();
    put_rows<(NPJ * 4 * NU + 255) / 256>(Vs, nullptr, 0, nvr, NPJ, dk);
    put_rows<(NPQ * 4 * NU + 255) / 256>(nullptr, Qt, LQ3, nqr, NPQ, dk);
    if (threadIdx.x < NPQ) Rs[threadIdx.x] = nrs;
    if (threadIdx.x < 3 * NPQ) Cs[threadIdx.x] = __expf(nm - nl);
    const bf16x8 fdo[2] = {nfdo[0], nfdo[1]};
    float pcur[3][4];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) pcur[t][r] = __uint_as_float((uint32_t)np[t][r] << 16);
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
          float g = a[t][r];
          if (p.p_drop > 0.f)
            g = attn_drop_keep(rng_key(seed, p.rng_stream), attn_drop_rowpairs(bh * p.T + i, p.T), j, p.p_drop) ? g * keep : 0.f;
          ds = pcur[t][r] * Cs[il * 3 + ((j >> 6) - kb0)] * (g - Rs[il]) * p.scale;
        }
        Dl[il * LDL + jl] = f2bf(ds);
      }
    // the p~ elements are consumed: the next iteration's loads overlap the dPpos MFMAs
    more = advance(b, ib0, len);
    if (more) fetch(b, ib0, len);
    __syncthreads();
    // dPpos[r0 + 16 w + m] += sum_i dS[i][(16 w + m) + i] Qv_i: A[m][k = i] = Dl[i][16 w + m + i]
    const int m = lane & 15, kq = 8 * (lane >> 4);
    bf16x8 fa;
#pragma unroll
    for (int e = 0; e < 8; ++e) fa[e] = (short)Dl[(kq + e) * LDL + 16 * w + m + kq + e];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const bf16x8 qb = *reinterpret_cast<const bf16x8*>(Qt + (16 * u + (lane & 15)) * LQ3 + kq);
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, qb, acc[u], 0, 0, 0);
    }
  }
#pragma unroll
  for (int u = 0; u < NU; ++u)
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

// ---------------------------------------------------------------------------------------------
// bwd2 kernel 2b: dK, dV as plain products over the saved bf16 dS and Pd (kernel 1 with SAVE):
//   dV[key] += sum_q Pd[q][key] dO[q],  dK[key] += sum_q dS[q][key] Qu[q]
// one workgroup per (b, h, 64 keys), 4 waves x 16 keys; per 64-query block the dO / Qu rows are staged
// [query][c] and the Pd / dS tiles [query][key] as copied (16-byte loads of 128-byte row runs), all four
// read TRANSPOSED into MFMA fragments (ds_read_b64_tr_b16).  No recompute of P, dP or the dropout mask.
// ---------------------------------------------------------------------------------------------
template <int NU>
__global__ __launch_bounds__(256, NU == 3 ? 2 : 1) void attn_bwd_dkv2_kernel(AbP p) {
  constexpr int LRK = 32 * (NU > 4 ? 4 : 2) + 8;   // row stride of the [query][c] images (head dim padded)
  __shared__ __attribute__((aligned(16))) uint16_t Os[BQ * LRK];     // dO block [query][c]
  __shared__ __attribute__((aligned(16))) uint16_t Qs[BQ * LRK];     // Qu block [query][c]
  __shared__ __attribute__((aligned(16))) uint16_t Pq[BQ * LW];     // Pd block [query][key]
  __shared__ __attribute__((aligned(16))) uint16_t Dq[BQ * LW];     // dS block [query][key]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const Blk3 blk = xcd_block3();
  const int64_t bh = blk.y;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int j0 = (int)blk.x * BK;
  const int len = p.lens ? (int)min<int64_t>(p.lens[b], p.T) : T;
  const int64_t hoff = h * p.dkh;
  zero_img<LRK>(Os, BQ);
  zero_img<LRK>(Qs, BQ);
  const int sbytes = (int)(p.B * p.H * p.T * p.ldt * 2);
  const __amdgpu_buffer_rsrc_t rds = __builtin_amdgcn_make_buffer_rsrc((void*)p.ds, (short)0, sbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rpd = __builtin_amdgcn_make_buffer_rsrc((void*)p.pdo, (short)0, sbytes, 0x00020000);
  f32x4 adv[NU], adk[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) { adv[u] = f32x4{0.f, 0.f, 0.f, 0.f}; adk[u] = adv[u]; }
  const int nqb = (j0 < len) ? (len + BQ - 1) / BQ : 0;
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4v;
  float4 ndo[NU], nqu[NU];
  u32x4v npd[2], nds[2];
  // query rows >= len and keys >= len read as 0 (key columns past len inside a written block are 0
  // already; whole rows >= len are dropped here)
  auto fetch = [&](int qb) {
    const int i0 = qb * BQ;
    fetch_rows<NU>(ndo, p.dO, p.ldq, b * p.T, i0, BQ, 0, len, hoff, dk);
    fetch_rows<NU>(nqu, p.qu, p.ldq, b * p.T, i0, BQ, 0, len, hoff, dk);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = threadIdx.x + 256 * q, row = c >> 3, c8 = c & 7;
      const int i = i0 + row, jc = j0 + 8 * c8;
      const uint32_t off = (i < len && jc < p.ldt) ? (uint32_t)(((bh * p.T + i) * p.ldt + jc) * 2) : AB_OOB;
      npd[q] = __builtin_amdgcn_raw_buffer_load_b128(rpd, off, 0, 0);
      nds[q] = __builtin_amdgcn_raw_buffer_load_b128(rds, off, 0, 0);
    }
  };
  if (nqb > 0) fetch(0);
  for (int qb = 0; qb < nqb; ++qb) {
    __syncthreads();
    put_rows<NU, LRK>(Os, nullptr, 0, ndo, BQ, dk);
    put_rows<NU, LRK>(Qs, nullptr, 0, nqu, BQ, dk);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = threadIdx.x + 256 * q, row = c >> 3, c8 = c & 7;
      *reinterpret_cast<u32x4v*>(Pq + row * LW + 8 * c8) = npd[q];
      *reinterpret_cast<u32x4v*>(Dq + row * LW + 8 * c8) = nds[q];
    }
    __syncthreads();
    if (qb + 1 < nqb) fetch(qb + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = tr_frag(Pq, LW, ks * 32, 16 * w, lane);   // A[key][q] = Pd[q][key]
      const bf16x8 da = tr_frag(Dq, LW, ks * 32, 16 * w, lane);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        adv[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, tr_frag(Os, LRK, ks * 32, 16 * u, lane), adv[u], 0, 0, 0);
        adk[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, tr_frag(Qs, LRK, ks * 32, 16 * u, lane), adk[u], 0, 0, 0);
      }
    }
  }
  const int jb = j0 + w * 16 + 4 * (lane >> 4);
#pragma unroll
  for (int u = 0; u < NU; ++u)
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
// bwd2 kernel 3b: per-chunk partials of dPpos[r] = sum_{b, i} dS[i][r - (T-1) + i] Qv_i over the saved bf16
// dS: per (h, 64 positions, batch chunk), query steps of 32 rows; the dS band [32][96] of the step is
// staged from HBM, the skewed A fragments and Qv^T read as kernel 3 does.
// ---------------------------------------------------------------------------------------------
template <int NU>
__global__ __launch_bounds__(256, NU == 3 ? 2 : 1) void attn_bwd_dpos2_kernel(AbP p) {
  __shared__ __attribute__((aligned(16))) uint16_t Dl[NPQ * LDL];    // dS [i - ib0][j - jbase]
  constexpr int DKP = 32 * (NU > 4 ? 4 : 2);
  __shared__ __attribute__((aligned(16))) uint16_t Qt[DKP * LQ3];    // Qv^T [c][i - ib0]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dkh;
  const int npos = 2 * T - 1;
  const Blk3 blk = xcd_block3();
  const int r0 = (int)blk.x * 64;
  const int64_t h = blk.y;
  const int64_t bchunk = blk.z;
  const int64_t hoff = h * p.dkh;
  for (int e = threadIdx.x; e < (DKP - dk) * LQ3; e += 256) Qt[dk * LQ3 + e] = 0;
  f32x4 acc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t b0 = bchunk * p.bpc;
  const int64_t b1 = min<int64_t>(p.B, b0 + p.bpc);
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
  constexpr int NE = NPQ * NPJ / 256;   // dS elements per thread per step
  float4 nqr[(NPQ * 4 * NU + 255) / 256];
  uint16_t nd[NE];
  auto fetch = [&](int64_t bb, int ib, int ln) {
    const int jb = r0 - (T - 1) + ib;
    const int64_t bhh = bb * p.H + h;
    fetch_rows<(NPQ * 4 * NU + 255) / 256>(nqr, p.qv, p.ldq, bb * p.T, ib, NPQ, 0, ln, hoff, dk);
#pragma unroll
    for (int it = 0; it < NE; ++it) {
      const int e = threadIdx.x + 256 * it;
      const int il = e / NPJ, jl = e - il * NPJ;
      const int i = ib + il, j = jb + jl;
      nd[it] = (i < ln && j >= 0 && j < ln) ? p.ds[(bhh * p.T + i) * p.ldt + j] : (uint16_t)0;
    }
  };
  int64_t b = b0;
  int ib0 = -NPQ, len = b0 < b1 ? ulen(b0) : 0;
  bool more = b0 < b1 && advance(b, ib0, len);
  if (more) fetch(b, ib0, len);
  while (more) {
    __syncthreads();
    put_rows<(NPQ * 4 * NU + 255) / 256>(nullptr, Qt, LQ3, nqr, NPQ, dk);
#pragma unroll
    for (int it = 0; it < NE; ++it) {
      const int e = threadIdx.x + 256 * it;
      const int il = e / NPJ, jl = e - il * NPJ;
      Dl[il * LDL + jl] = nd[it];
    }
    __syncthreads();
    more = advance(b, ib0, len);
    if (more) fetch(b, ib0, len);
    // dPpos[r0 + 16 w + m] += sum_i dS[i][(16 w + m) + i] Qv_i: A[m][k = i] = Dl[i][16 w + m + i]
    const int m = lane & 15, kq = 8 * (lane >> 4);
    bf16x8 fa;
#pragma unroll
    for (int e = 0; e < 8; ++e) fa[e] = (short)Dl[(kq + e) * LDL + 16 * w + m + kq + e];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const bf16x8 qb = *reinterpret_cast<const bf16x8*>(Qt + (16 * u + (lane & 15)) * LQ3 + kq);
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, qb, acc[u], 0, 0, 0);
    }
  }
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = r0 + 16 * w + 4 * (lane >> 4) + r, c = 16 * u + (lane & 15);
      if (rr < npos && c < dk) p.dpos_part[(bchunk * npos + rr) * p.d + hoff + c] = acc[u][r];
    }
}

constexpr int DPOS_MAX_CHUNKS = 64;   // dPpos partials: one chunk per utterance (up to 64)

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_relpos_attn_bwd_ws(int64_t B, int64_t H, int64_t T, int64_t d) {
  return B * H * T + (B < kdfm::DPOS_MAX_CHUNKS ? B : (int64_t)kdfm::DPOS_MAX_CHUNKS) * (2 * T - 1) * d;
}

int kdfm_relpos_attn_bwd(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                         const float* pos, const float* lse, const uint16_t* p_tilde, const float* m_blk,
                         const int64_t* lengths, float* dqu, float* dqv, float* dqkv, float* dpos,
                         float* ws, int64_t ws_len, int64_t B, int64_t H, int64_t T, int64_t d, float scale,
                         float dropout_p, const uint64_t* seed, uint64_t rng_stream, void* stream) {
  return kdfm_relpos_attn_bwd_parts(dO, O, qu, qv, qkv, pos, lse, p_tilde, m_blk, lengths, dqu, dqv, dqkv, dpos, ws, ws_len, B, H, T, d,
                                    scale, dropout_p, seed, rng_stream, KDFM_ATTN_BWD_ALL, stream);
}

int kdfm_relpos_attn_bwd_parts(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                               const float* pos, const float* lse, const uint16_t* p_tilde, const float* m_blk,
                               const int64_t* lengths, float* dqu, float* dqv, float* dqkv, float* dpos, float* ws, int64_t ws_len, int64_t B, int64_t H, int64_t T,
                               int64_t d, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                               int32_t parts, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dO && O && qu && qv && qkv && pos && lse && ws, "null pointer");
  KDFM_REQUIRE(!(parts & KDFM_ATTN_BWD_DQ) || (dqu && dqv), "dq part needs dqu / dqv");
  KDFM_REQUIRE(!(parts & KDFM_ATTN_BWD_DKV) || dqkv, "dkv part needs dqkv");
  KDFM_REQUIRE(!(parts & KDFM_ATTN_BWD_DPOS) || dpos, "dpos part needs dpos");
  KDFM_REQUIRE(!(parts & (KDFM_ATTN_BWD_DKV | KDFM_ATTN_BWD_DPOS)) || (p_tilde && m_blk),
               "dkv / dpos parts need the forward's p_tilde and m_blk");
  KDFM_REQUIRE(H > 0 && d % H == 0, "d must be a multiple of H");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk <= 64 && dk % 4 == 0, "head dim must be a multiple of 4 and <= 64");
  const bool wide = dk > 48;   // 4 output column tiles of 16 (FastConformer's 64) instead of 3
  KDFM_REQUIRE(T > 0 && T <= 4096 && d % 4 == 0, "bad T / d");
  KDFM_REQUIRE(dropout_p == 0.f || seed, "dropout needs a seed");
  KDFM_REQUIRE(ws_len >= kdfm_relpos_attn_bwd_ws(B, H, T, d), "workspace too small (kdfm_relpos_attn_bwd_ws)");
  KDFM_REQUIRE((((uintptr_t)dO | (uintptr_t)qu | (uintptr_t)qv | (uintptr_t)qkv | (uintptr_t)pos) & 15) == 0,
               "operands must be 16-byte aligned");
  if (B == 0) return KDFM_OK;
  AbP p{};
  p.dO = dO; p.qu = qu; p.qv = qv; p.k = qkv + d; p.v = qkv + 2 * d; p.pos = pos; p.lse = lse; p.pt = p_tilde; p.mblk = m_blk;
  p.lens = lengths;
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
    if (wide)
      hipLaunchKernelGGL(attn_bwd_dq_kernel<4>, dim3((unsigned)ceil_div(T, BQ), (unsigned)(B * H)), dim3(256), 0, st, p);
    else
      hipLaunchKernelGGL(attn_bwd_dq_kernel<3>, dim3((unsigned)ceil_div(T, BQ), (unsigned)(B * H)), dim3(256), 0, st, p);
    rc = check_launch("kdfm_relpos_attn_bwd(dq)");
    if (rc) return rc;
  }
  if (parts & KDFM_ATTN_BWD_DKV) {
    if (wide)
      hipLaunchKernelGGL(attn_bwd_dkv_kernel<4>, dim3((unsigned)ceil_div(T, BK), (unsigned)(B * H)), dim3(256), 0, st, p);
    else
      hipLaunchKernelGGL(attn_bwd_dkv_kernel<3>, dim3((unsigned)ceil_div(T, BK), (unsigned)(B * H)), dim3(256), 0, st, p);
    rc = check_launch("kdfm_relpos_attn_bwd(dkv)");
    if (rc) return rc;
  }
  if (!(parts & KDFM_ATTN_BWD_DPOS)) return KDFM_OK;
  const int64_t npos = 2 * T - 1;
  if (wide)
    hipLaunchKernelGGL(attn_bwd_dpos_kernel<4>, dim3((unsigned)ceil_div(npos, 64), (unsigned)H, (unsigned)chunks),
                       dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(attn_bwd_dpos_kernel<3>, dim3((unsigned)ceil_div(npos, 64), (unsigned)H, (unsigned)chunks),
                       dim3(256), 0, st, p);
  rc = check_launch("kdfm_relpos_attn_bwd(dpos)");
  if (rc) return rc;
  hipLaunchKernelGGL(attn_dpos_fold_kernel, dim3((unsigned)ceil_div(npos * d, 256)), dim3(256), 0, st, p.dpos_part,
                     dpos, npos * d, chunks);
  return check_launch("kdfm_relpos_attn_bwd(fold)");
}

int64_t kdfm_relpos_attn_bwd2_ldt(int64_t T) { return kdfm::ceil_div(T, 8) * 8; }

int64_t kdfm_relpos_attn_bwd2_dpos_ws(int64_t B, int64_t T, int64_t d) {
  return (B < kdfm::DPOS_MAX_CHUNKS ? B : (int64_t)kdfm::DPOS_MAX_CHUNKS) * (2 * T - 1) * d;
}

namespace kdfm {
namespace {
int ab2_setup(AbP& p, const float* qu, const float* qv, const float* qkv, const float* lse, const int64_t* lengths,
              int64_t B, int64_t H, int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed,
              uint64_t rng_stream) {
  KDFM_REQUIRE(H > 0 && d % H == 0, "d must be a multiple of H");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk <= 128 && dk % 4 == 0, "head dim must be a multiple of 4 and <= 128");
  KDFM_REQUIRE(T > 0 && T <= 4096 && d % 4 == 0, "bad T / d");
  KDFM_REQUIRE(dropout_p == 0.f || seed, "dropout needs a seed");
  KDFM_REQUIRE(B * H * T * kdfm_relpos_attn_bwd2_ldt(T) * 2 < (1ll << 31), "dS / Pd larger than 2 GiB (buffer offsets)");
  p = AbP{};
  p.qu = qu; p.qv = qv; p.k = qkv ? qkv + d : nullptr; p.v = qkv ? qkv + 2 * d : nullptr; p.lse = lse;
  p.lens = lengths;
  p.B = B; p.H = H; p.T = T; p.d = d; p.dkh = dk; p.ldq = d; p.ldkv = 3 * d;
  p.scale = scale; p.p_drop = dropout_p; p.seed = seed; p.rng_stream = rng_stream;
  p.ldt = kdfm_relpos_attn_bwd2_ldt(T);
  const int chunks = (int)(B < DPOS_MAX_CHUNKS ? B : DPOS_MAX_CHUNKS);
  p.bpc = B > 0 ? (int)ceil_div(B, chunks) : 1;
  return KDFM_OK;
}
}  // namespace
}  // namespace kdfm

int kdfm_relpos_attn_bwd2_dq(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                             const float* pos, const float* lse, const int64_t* lengths, float* rsum, uint16_t* ds,
                             uint16_t* pd, float* dqu, float* dqv, int64_t B, int64_t H, int64_t T, int64_t d,
                             float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dO && O && qu && qv && qkv && pos && lse && ds && pd && dqu && dqv, "null pointer");
  KDFM_REQUIRE((((uintptr_t)dO | (uintptr_t)O | (uintptr_t)qu | (uintptr_t)qv | (uintptr_t)qkv | (uintptr_t)pos |
                 (uintptr_t)ds | (uintptr_t)pd) & 15) == 0, "operands must be 16-byte aligned");
  KDFM_REQUIRE(B * T * 3 * d * 4 < (1ll << 31), "qkv larger than 2 GiB (buffer offsets)");
  AbP p;
  int rc = ab2_setup(p, qu, qv, qkv, lse, lengths, B, H, T, d, scale, dropout_p, seed, rng_stream);
  if (rc || B == 0) return rc;
  p.dO = dO; p.pos = pos; p.rsum = rsum; p.dqu = dqu; p.dqv = dqv; p.ds = ds; p.pdo = pd; p.O = O;
  hipStream_t st = as_stream(stream);
  if (p.dkh > 64)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<8, true, true>), dim3((unsigned)ceil_div(T, BQ), (unsigned)(B * H)), dim3(256), 0, st, p);
  else if (p.dkh > 48)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<4, true, true>), dim3((unsigned)ceil_div(T, BQ), (unsigned)(B * H)), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<3, true, true>), dim3((unsigned)ceil_div(T, BQ), (unsigned)(B * H)), dim3(256), 0, st, p);
  return check_launch("kdfm_relpos_attn_bwd2_dq");
}

int kdfm_relpos_attn_bwd2_dq3(const float* dO, const float* O, const float* qu, const float* qv, const uint16_t* kb,
                              const uint16_t* vb, const float* centre, const uint16_t* pb, const float* lse,
                              const int64_t* lengths, uint16_t* ds, uint16_t* pd, float* dqu, float* dqv, int64_t B,
                              int64_t H, int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed,
                              uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dO && O && qu && qv && kb && vb && centre && pb && lse && ds && pd && dqu && dqv, "null pointer");
  KDFM_REQUIRE((((uintptr_t)dO | (uintptr_t)O | (uintptr_t)qu | (uintptr_t)qv | (uintptr_t)kb | (uintptr_t)vb |
                 (uintptr_t)pb | (uintptr_t)ds | (uintptr_t)pd) & 15) == 0, "operands must be 16-byte aligned");
  AbP p;
  int rc = ab2_setup(p, qu, qv, nullptr, lse, lengths, B, H, T, d, scale, dropout_p, seed, rng_stream);
  if (rc || B == 0) return rc;
  p.dO = dO; p.dqu = dqu; p.dqv = dqv; p.ds = ds; p.pdo = pd; p.O = O;
  p.kb = kb; p.vb = vb; p.cen = centre; p.pb = pb; p.Tp = attn_prep_tp(T); p.npb = attn_prep_npb(T);
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)ceil_div(T, BQ), (unsigned)(B * H));
  if (p.dkh > 64)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<8, true, true, true>), grid, dim3(256), 0, st, p);
  else if (p.dkh > 48)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<4, true, true, true>), grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<3, true, true, true>), grid, dim3(256), 0, st, p);
  return check_launch("kdfm_relpos_attn_bwd2_dq3");
}

int kdfm_relpos_attn_bwd2_dkv(const float* dO, const float* qu, const uint16_t* ds, const uint16_t* pd,
                              const int64_t* lengths, float* dqkv, int64_t B, int64_t H, int64_t T, int64_t d,
                              void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dO && qu && ds && pd && dqkv, "null pointer");
  KDFM_REQUIRE((((uintptr_t)dO | (uintptr_t)qu | (uintptr_t)ds | (uintptr_t)pd) & 15) == 0,
               "operands must be 16-byte aligned");
  AbP p;
  int rc = ab2_setup(p, qu, nullptr, nullptr, nullptr, lengths, B, H, T, d, 1.f, 0.f, nullptr, 0);
  if (rc || B == 0) return rc;
  p.dO = dO; p.ds = const_cast<uint16_t*>(ds); p.pdo = const_cast<uint16_t*>(pd);
  p.dk = dqkv + d; p.dv = dqkv + 2 * d;
  hipStream_t st = as_stream(stream);
  if (p.dkh > 64)
    hipLaunchKernelGGL(attn_bwd_dkv2_kernel<8>, dim3((unsigned)ceil_div(T, BK), (unsigned)(B * H)), dim3(256), 0, st, p);
  else if (p.dkh > 48)
    hipLaunchKernelGGL(attn_bwd_dkv2_kernel<4>, dim3((unsigned)ceil_div(T, BK), (unsigned)(B * H)), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(attn_bwd_dkv2_kernel<3>, dim3((unsigned)ceil_div(T, BK), (unsigned)(B * H)), dim3(256), 0, st, p);
  return check_launch("kdfm_relpos_attn_bwd2_dkv");
}

int kdfm_relpos_attn_bwd2_dpos(const float* qv, const uint16_t* ds, const int64_t* lengths, float* dpos, float* ws,
                               int64_t ws_len, int64_t B, int64_t H, int64_t T, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(qv && ds && dpos && ws, "null pointer");
  KDFM_REQUIRE(ws_len >= kdfm_relpos_attn_bwd2_dpos_ws(B, T, d), "workspace too small (kdfm_relpos_attn_bwd2_dpos_ws)");
  AbP p;
  int rc = ab2_setup(p, nullptr, qv, nullptr, nullptr, lengths, B, H, T, d, 1.f, 0.f, nullptr, 0);
  if (rc || B == 0) return rc;
  p.ds = const_cast<uint16_t*>(ds); p.dpos_part = ws;
  const int chunks = (int)(B < DPOS_MAX_CHUNKS ? B : DPOS_MAX_CHUNKS);
  const int64_t npos = 2 * T - 1;
  hipStream_t st = as_stream(stream);
  if (p.dkh > 64)
    hipLaunchKernelGGL(attn_bwd_dpos2_kernel<8>, dim3((unsigned)ceil_div(npos, 64), (unsigned)H, (unsigned)chunks),
                       dim3(256), 0, st, p);
  else if (p.dkh > 48)
    hipLaunchKernelGGL(attn_bwd_dpos2_kernel<4>, dim3((unsigned)ceil_div(npos, 64), (unsigned)H, (unsigned)chunks),
                       dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(attn_bwd_dpos2_kernel<3>, dim3((unsigned)ceil_div(npos, 64), (unsigned)H, (unsigned)chunks),
                       dim3(256), 0, st, p);
  rc = check_launch("kdfm_relpos_attn_bwd2_dpos");
  if (rc) return rc;
  hipLaunchKernelGGL(attn_dpos_fold_kernel, dim3((unsigned)ceil_div(npos * d, 256)), dim3(256), 0, st, p.dpos_part,
                     dpos, npos * d, chunks);
  return check_launch("kdfm_relpos_attn_bwd2_dpos(fold)");
}

}  // extern "C"
