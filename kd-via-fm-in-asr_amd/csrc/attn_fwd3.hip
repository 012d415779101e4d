// Relative-position MHA forward over PREPARED bf16 operands (the single-pass / lse-only form the bwd2 backward
// and inference use): the operands, MFMAs and counter-RNG dropout mask of relpos_attn_fwd_kernel<false, NU, false>
// (attn_fused.hip) with the online softmax in the exp2 domain (O within 1e-3, lse within 2e-6 of that kernel's),
// restaged for occupancy:
//   * kdfm_attn_kv_prep writes each utterance's centred keys / values (attn_centre.h) ONCE as bf16 tiles
//     [b, h][key][c] with the LDS row stride (head dim padded to 48 / 64 / 128, + 8), and the value centre;
//     kdfm_attn_band_prep every layer's projected positions as bf16 rows [layer, h][64 + r][c] with zero rows
//     around them.  Every operand tile of a (64 queries, 64 keys) step is then ONE contiguous byte range
//     (K 64 rows, V 64 rows, the Ppos band 128 rows from r = T-1-(i0+63)+j0), copied into LDS by LDS-DMA
//     (global_load_lds_dwordx4, 1 KB per wave-instruction): no staging registers, no conversion, no
//     ds_write pass (the register-staged kernel spent ~30 % of a key block there, profiles/r03/final_attn_probe.log).
//   * rel_shift as lane permutes: S_bd[ii][jj] = G[ii][jj - ii + 15] is read from the MFMA accumulators of G =
//     Qv Pband^T with ds_bpermute (5 per row register) instead of an f32 G tile written to and read back from
//     LDS (20.7 KB per workgroup and two wave syncs per key block).
//   * P V reads V [key][c] transposed (ds_read_b64_tr_b16) instead of a transposed V^T image.
//   * each wave's P^T tile [64 keys][16 rows] goes into the band region once the score MFMAs have read it.
// LDS per workgroup (K | V | band): 28 KB at head dim <= 48 (4 workgroups, 16 waves per CU, 117 registers),
// 36 KB at <= 64, 68 KB at 128 (the register-staged kernel: 67 KB, 2 workgroups).
#include "gemm_common.h"
#include "attn_centre.h"

namespace kdfm {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t3;
typedef __attribute__((address_space(1))) void gl_void_t3;
typedef short v4s3 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s3 lds_v4s3;

constexpr int A3Q = 64;            // queries per workgroup (4 waves x 16)
constexpr int A3K = 64;            // keys per step
constexpr int A3BAND = 128;        // Ppos band rows staged per step (127 used)
constexpr int A3PAD0 = kAttnBandPad0;   // zero rows before the first position row of a prepared band
constexpr int A3LDT = 16;          // bf16 row stride of the per-wave P^T tile [64 keys][16 rows]

template <int NU> struct A3Geo {
  static constexpr int DKP = NU == 3 ? 48 : NU > 4 ? 128 : 64;   // padded head dim (attn_prep_dkp)
  static constexpr int KS = DKP / 32;              // 32-wide MFMA k-steps over it ...
  static constexpr bool TAIL = DKP % 32 != 0;      // ... and one 16-wide (v_mfma_f32_16x16x16_bf16) at 48
  static constexpr int LR = DKP + 8;               // bf16 row stride (8-byte aligned transposed reads)
  static constexpr int KCH = A3K * LR * 2 / 1024;  // 1 KB DMA chunks per K / V tile
  static constexpr int BCH = A3BAND * LR * 2 / 1024;
  static_assert(A3K * LR * 2 % 1024 == 0 && A3BAND * LR * 2 % 1024 == 0, "tiles must be whole 1 KB chunks");
};

__host__ __device__ inline int a3_dkp(int64_t dk) { return attn_prep_dkp(dk); }
__host__ __device__ inline int64_t a3_tp(int64_t T) { return attn_prep_tp(T); }
__host__ __device__ inline int64_t a3_npb(int64_t T) { return attn_prep_npb(T); }

// ---- preparation --------------------------------------------------------------------------------------
// kb / vb [b*H + h][Tp][LR]: rows j < T hold bf16(K_j - kc) / bf16(V_j - vc) in columns < dk, zeros elsewhere;
// cen [b*H + h][2][DKP] = (kc, vc) f32 (zeros past dk).  One workgroup per (64 rows, utterance b, hpw (kind,
// head) tiles): the centres of its tiles (one thread per float4 column group summing the utterance's first n rows
// in order -- attn_centre.h's kv_centre arithmetic, the same bits), then the 64 rows' conversion, one (kind, head)
// tile after the other with the next tile's loads issued before the current one is converted (and the first
// tile's before the centres).  A thread owns fixed (row, 8-column group) items of every tile: compile-time
// index arithmetic, PER x 2 float4 loads in flight per tile.
template <int DKP>
__global__ __launch_bounds__(256) void attn_kv_prep_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ lens,
                                                           uint16_t* __restrict__ kb, uint16_t* __restrict__ vb,
                                                           float* __restrict__ cen, int64_t H, int T, int64_t d, int dk,
                                                           int64_t Tp, int hpw) {
  constexpr int LR = DKP + 8, P8 = LR / 8, ITEMS = 64 * P8, PER = (ITEMS + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) float Cn[];   // [kind][head][DKP]
  const int64_t b = blockIdx.y;
  const int Hh = (int)H;
  const int kh0 = blockIdx.z * hpw, kh1 = min(2 * Hh, kh0 + hpw);   // this workgroup's (kind, head) tiles
  const int len = lens ? (int)min<int64_t>(lens[b], T) : T;
  const float* kbase = qkv + b * T * 3 * d + d;   // row 0 of utterance b, K columns (V at + d)
  const int j0 = blockIdx.x * 64;
  int rowoff[PER], c0q[PER];
  float m0q[PER], m1q[PER];
  bool itq[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int item = threadIdx.x + 256 * q;
    itq[q] = item < ITEMS;
    const int rr = item / P8, c0 = (item - rr * P8) * 8;
    const int j = j0 + rr;
    rowoff[q] = (j < T ? j : 0);
    c0q[q] = c0;
    m0q[q] = (j < T && c0 < dk) ? 1.f : 0.f;
    m1q[q] = (j < T && c0 + 4 < dk) ? 1.f : 0.f;
  }
  auto load = [&](int kh, float4 (&a)[PER], float4 (&e)[PER]) {
    const int kind = kh >= Hh ? 1 : 0, h = kh - kind * Hh;
    const float* src = kbase + (int64_t)kind * d + (int64_t)h * dk;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const float* rs = src + (int64_t)rowoff[q] * 3 * d;
      const int c0 = c0q[q];
      a[q] = itq[q] ? *reinterpret_cast<const float4*>(rs + (c0 < dk ? c0 : 0)) : make_float4(0.f, 0.f, 0.f, 0.f);
      e[q] = itq[q] ? *reinterpret_cast<const float4*>(rs + (c0 + 4 < dk ? c0 + 4 : 0)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  float4 a0[PER], e0[PER];
  load(kh0, a0, e0);
  // centres
  const int n = len >= 16 ? 16 : len >= 8 ? 8 : len >= 4 ? 4 : len >= 2 ? 2 : (len > 0 ? 1 : 0);
  const float inv = n > 0 ? 1.f / (float)n : 0.f;   // a power of two: exact
  const int nkh = kh1 - kh0;
  for (int e = threadIdx.x; e < nkh * DKP; e += 256) Cn[e] = 0.f;
  __syncthreads();
  const int cq = dk >> 2;
  for (int g = threadIdx.x; g < nkh * cq; g += 256) {   // (kind, head, float4 column group)
    const int kl = g / cq, c4 = (g - kl * cq) * 4, kh = kh0 + kl;
    const int kind = kh >= Hh ? 1 : 0, h = kh - kind * Hh;
    const float* src = kbase + (int64_t)kind * d + (int64_t)h * dk + c4;
    float4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = *reinterpret_cast<const float4*>(src + (int64_t)(r < n ? r : 0) * 3 * d);
    float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float m = r < n ? 1.f : 0.f;
      sm.x += m * v[r].x; sm.y += m * v[r].y; sm.z += m * v[r].z; sm.w += m * v[r].w;
    }
    float* o = Cn + kl * DKP + c4;
    o[0] = sm.x * inv; o[1] = sm.y * inv; o[2] = sm.z * inv; o[3] = sm.w * inv;
  }
  __syncthreads();
  if (blockIdx.x == 0)
    for (int e = threadIdx.x; e < nkh * DKP; e += 256) {   // cen[(b H + h)][kind][c]
      const int kl = e / DKP, c = e - kl * DKP, kh = kh0 + kl;
      const int kind = kh >= Hh ? 1 : 0, h = kh - kind * Hh;
      cen[((b * H + h) * 2 + kind) * DKP + c] = Cn[e];
    }
  for (int kh = kh0; kh < kh1; ++kh) {
    float4 a1[PER], e1[PER];
    if (kh + 1 < kh1) load(kh + 1, a1, e1);
    const int kind = kh >= Hh ? 1 : 0, h = kh - kind * Hh;
    const float* cc = Cn + (kh - kh0) * DKP;
    uint16_t* dst = (kind ? vb : kb) + ((b * H + h) * Tp + j0) * LR;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (!itq[q]) continue;
      const int item = threadIdx.x + 256 * q;
      const int c0 = c0q[q];
      const float4 a = a0[q], e = e0[q];
      const float m0 = m0q[q], m1 = m1q[q];
      const int ca = c0 < DKP ? c0 : 0, cb = c0 + 4 < DKP ? c0 + 4 : 0;
      // (a - c) * m: the subtraction is the register-staged kernel's rk - ck, rounded to bf16 by the same RNE
      const float t[8] = {(a.x - cc[ca]) * m0, (a.y - cc[ca + 1]) * m0, (a.z - cc[ca + 2]) * m0, (a.w - cc[ca + 3]) * m0,
                          (e.x - cc[cb]) * m1, (e.y - cc[cb + 1]) * m1, (e.z - cc[cb + 2]) * m1, (e.w - cc[cb + 3]) * m1};
      *reinterpret_cast<bf16x8*>(dst + item * 8) = pack_bf16x8<bf16x8>(t);   // row item / P8, column c0
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) { a0[q] = a1[q]; e0[q] = e1[q]; }
  }
}

// pb [layer*H + h][NPB][LR]: row A3PAD0 + r = bf16(pos[layer][r][h*dk + c]) (c < dk), zeros elsewhere
template <int DKP>
__global__ __launch_bounds__(256) void attn_band_prep_kernel(const float* __restrict__ pos, int64_t ld_layer,
                                                             uint16_t* __restrict__ pb, int64_t H, int64_t npos,
                                                             int64_t d, int dk, int64_t npb) {
  constexpr int LR = DKP + 8, P8 = LR / 8;
  const int64_t lh = blockIdx.y, l = lh / H, h = lh - l * H;
  const int64_t R0 = (int64_t)blockIdx.x * 64;
  for (int e = threadIdx.x; e < 64 * P8; e += 256) {
    const int rr = e / P8, c0 = (e - rr * P8) * 8;
    const int64_t R = R0 + rr, r = R - A3PAD0;
    if (R >= npb) continue;
    const bool in = r >= 0 && r < npos;
    const float* src = pos + l * ld_layer + (in ? r : 0) * d + h * dk;
    const float m0 = (in && c0 < dk) ? 1.f : 0.f, m1 = (in && c0 + 4 < dk) ? 1.f : 0.f;
    const float4 a = *reinterpret_cast<const float4*>(src + (c0 < dk ? c0 : 0));
    const float4 q = *reinterpret_cast<const float4*>(src + (c0 + 4 < dk ? c0 + 4 : 0));
    const float t[8] = {a.x * m0, a.y * m0, a.z * m0, a.w * m0, q.x * m1, q.y * m1, q.z * m1, q.w * m1};
    *reinterpret_cast<bf16x8*>(pb + (lh * npb + R) * LR + c0) = pack_bf16x8<bf16x8>(t);
  }
}

// ---- the forward --------------------------------------------------------------------------------------
struct Attn3P {
  const float* qu; const float* qv; const uint16_t* kb; const uint16_t* vb; const float* cen; const uint16_t* pb;
  const int64_t* lens;
  float* o; float* lse;
  int64_t B, H, T, d, dk, Tp, npb;
  float scale, p_drop;
  const uint64_t* seed; uint64_t rng_stream;
};

__device__ __forceinline__ bf16x8 a3_frag8(const float* head, int c0, int valid) {
  const float m0 = valid >= 4 ? 1.f : 0.f, m1 = valid >= 8 ? 1.f : 0.f;
  const float4 a = *reinterpret_cast<const float4*>(head + (valid >= 4 ? c0 : 0));
  const float4 b = *reinterpret_cast<const float4*>(head + (valid >= 8 ? c0 + 4 : 0));
  const float t[8] = {a.x * m0, a.y * m0, a.z * m0, a.w * m0, b.x * m1, b.y * m1, b.z * m1, b.w * m1};
  return pack_bf16x8<bf16x8>(t);
}

typedef short bf16x4 __attribute__((ext_vector_type(4)));
// 4 consecutive bf16 of a row (the 16-wide tail k-step); columns at or past `valid` read as 0
__device__ __forceinline__ bf16x4 a3_frag4(const float* head, int c0, int valid) {
  const float m = valid >= 4 ? 1.f : 0.f;
  const float4 a = *reinterpret_cast<const float4*>(head + (valid >= 4 ? c0 : 0));
  const uint32_t lo = pack_bf16x2(a.x * m, a.y * m), hi = pack_bf16x2(a.z * m, a.w * m);
  return __builtin_bit_cast(bf16x4, make_uint2(lo, hi));
}

// B operand X[k][n] read transposed out of a [k][n] bf16 LDS image (attn_bwd.hip tr_frag)
__device__ __forceinline__ bf16x8 a3_tr_frag(const uint16_t* img, int ld, int k0, int n0, int lane) {
  const int li = lane & 15;
  const uint16_t* a = img + (k0 + 8 * (lane >> 4) + (li >> 2)) * ld + n0 + 4 * (li & 3);
  const v4s3 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s3*)a);
  const v4s3 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s3*)(a + 4 * ld));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int CTRL>
__device__ __forceinline__ float a3_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float a3_max16(float v) {
  v = fmaxf(v, a3_dpp<0xB1>(v));
  v = fmaxf(v, a3_dpp<0x4E>(v));
  v = fmaxf(v, a3_dpp<0x141>(v));
  return fmaxf(v, a3_dpp<0x140>(v));
}
// the row max over the 16 lanes of each of the four C-tile rows at once: 16 DPP max instructions (the builtin
// form costs a v_mov_dpp and a canonicalising v_max per stage, 48).  The leading s_nop covers the DPP read-
// after-VALU-write hazard of the inputs; within the block each register's next DPP read is 4 instructions
// after its write.
__device__ __forceinline__ void a3_max16x4(float& a, float& b, float& c, float& d) {
  asm volatile(
      "s_nop 1\n"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %3, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %2, %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %3, %3, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %2, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %3, %3, %3 row_half_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %2, %2, %2 row_mirror row_mask:0xf bank_mask:0xf\n"
      "v_max_f32_dpp %3, %3, %3 row_mirror row_mask:0xf bank_mask:0xf\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ float a3_sum16(float v) {
  v += a3_dpp<0xB1>(v);
  v += a3_dpp<0x4E>(v);
  v += a3_dpp<0x141>(v);
  return v + a3_dpp<0x140>(v);
}

template <int NU>
__global__ __launch_bounds__(256, NU == 3 ? 4 : NU == 4 ? 3 : 2) void relpos_attn_fwd3_kernel(Attn3P p) {
  using Gm = A3Geo<NU>;
  constexpr int KS = Gm::KS, LR = Gm::LR, KCH = Gm::KCH, BCH = Gm::BCH, NCH = 2 * KCH + BCH;
  // K tile | V tile | band rows, contiguous (wave w's DMA chunks at fixed offsets).  The per-wave P^T tiles
  // [key][row] reuse the band tile once every wave has read it (a barrier after the score MFMAs): 28 KB per
  // workgroup at head dim <= 48 (row stride 56), 4 workgroups per CU
  static_assert(4 * A3K * A3LDT <= A3BAND * LR, "the P^T tiles must fit in the band tile");
  __shared__ __attribute__((aligned(16))) uint16_t Sm[(2 * A3K + A3BAND) * LR];
  uint16_t* const Ks = Sm;
  uint16_t* const Vs = Sm + A3K * LR;
  uint16_t* const Pr = Sm + 2 * A3K * LR;

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int T = (int)p.T, dk = (int)p.dk;
  const Blk3 blk = xcd_block3();
  const int64_t bh = blk.y;
  const int64_t b = bh / p.H, h = bh - b * p.H;
  const int i0 = (int)blk.x * A3Q;
  const int len = p.lens ? (int)p.lens[b] : T;
  const int lim = min(len, T);
  const int nkb = (lim + A3K - 1) / A3K;
  const int64_t hoff = h * p.dk;
  const uint4* ksrc = reinterpret_cast<const uint4*>(p.kb + bh * p.Tp * LR);
  const uint4* vsrc = reinterpret_cast<const uint4*>(p.vb + bh * p.Tp * LR);
  const uint16_t* bsrc = p.pb + h * p.npb * LR;

  // one key step's operands: K rows [j0, j0 + 64), V rows, band rows [rbase, rbase + 128) of the prepared
  // band (row A3PAD0 + r holds position r) -- NCH 1 KB chunks, wave w takes chunks w, w + 4, ...
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const uint32_t loff = (uint32_t)lane * 16u;
  auto issue = [&](int j0) {
    // wave wu copies chunks wu, wu + 4, ... of each tile: uniform (SGPR) chunk addresses plus this lane's 16
    // bytes, LDS destinations at compile-time offsets from the wave's first chunk
    const int rb = T - 1 - (i0 + A3Q - 1) + j0 + A3PAD0;
    const char* kbase = reinterpret_cast<const char*>(ksrc) + (int64_t)j0 * LR * 2 + wu * 1024;
    const char* vbase = reinterpret_cast<const char*>(vsrc) + (int64_t)j0 * LR * 2 + wu * 1024;
    const char* bbase = reinterpret_cast<const char*>(bsrc + (int64_t)rb * LR) + wu * 1024;
    uint4* const ld0 = reinterpret_cast<uint4*>(Sm) + wu * 64;
#pragma unroll
    for (int i = 0; i < (KCH + 3) / 4; ++i)
      if (4 * i + 3 < KCH || wu + 4 * i < KCH) {
        __builtin_amdgcn_global_load_lds((gl_void_t3*)(kbase + i * 4096 + loff), (lds_void_t3*)(ld0 + i * 256), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gl_void_t3*)(vbase + i * 4096 + loff), (lds_void_t3*)(ld0 + KCH * 64 + i * 256),
                                         16, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < (BCH + 3) / 4; ++i)
      if (4 * i + 3 < BCH || wu + 4 * i < BCH)
        __builtin_amdgcn_global_load_lds((gl_void_t3*)(bbase + i * 4096 + loff),
                                         (lds_void_t3*)(ld0 + 2 * KCH * 64 + i * 256), 16, 0, 0);
  };
  if (nkb > 0) issue(0);

  // this lane's query row (A-fragment row): Qu / Qv fragments
  const int iq = i0 + w * 16 + (lane & 15);
  bf16x8 fu[KS], fv[KS];
  bf16x4 fut = {}, fvt = {};   // the 16-wide tail step (TAIL): columns 32 KS + 4 (lane >> 4) .. + 3
  {
    const int64_t off = (b * p.T + (iq < T ? iq : 0)) * p.d + hoff;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = ks * 32 + 8 * (lane >> 4);
      const int valid = (iq < T) ? dk - c0 : 0;
      fu[ks] = a3_frag8(p.qu + off, c0, valid);
      fv[ks] = a3_frag8(p.qv + off, c0, valid);
    }
    if constexpr (Gm::TAIL) {
      const int c0 = KS * 32 + 4 * (lane >> 4);
      const int valid = (iq < T) ? dk - c0 : 0;
      fut = a3_frag4(p.qu + off, c0, valid);
      fvt = a3_frag4(p.qv + off, c0, valid);
    }
  }
  const int q4 = lane >> 4, lo = lane & 15;
  const int ib = i0 + w * 16 + 4 * q4;   // C-layout rows ib + r
  // online softmax state in the exp2 domain: m2 = running row max of s * scale * log2(e); per-LANE partial
  // sums of exp2(s * sl2 - m2) (and of the dropped-out probabilities), reduced over the row's 16 lanes once
  // after the loop (the row max is reduced every step -- the rescale needs it)
  const float sl2 = p.scale * 1.4426950408889634f;
  float m2[4], lsum[4], psum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m2[r] = -3.0e38f; lsum[r] = 0.f; psum[r] = 0.f; }
  // rel_shift permute per row register r: S_bd(t, r) = G[t + (off >= 16)][r] of lane (off & 15) + 16 q4
  int bsrc_lane[4];
  bool bhi[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int off = lo - 4 * q4 - r + 15;   // 0 .. 30
    bsrc_lane[r] = ((off & 15) + 16 * q4) * 4;
    bhi[r] = off >= 16;
  }

  const uint64_t seed = (p.p_drop > 0.f) ? load_seed(p.seed) : 0ull;
  const uint64_t dkey = rng_key(seed, p.rng_stream);
  const float keep_scale = (p.p_drop > 0.f) ? 1.f / (1.f - p.p_drop) : 1.f;
  const bool drop = p.p_drop > 0.f;
  const uint32_t thr = drop_threshold(p.p_drop);
  // dropout (common.h attn_drop_keep): keys 16 t + lo and 16 t + (lo ^ 1) share one pair hash, so this lane
  // hashes two of its four rows (even lanes rows ib, ib + 1; odd lanes ib + 2, ib + 3) and takes the other
  // two from its pair partner (DPP swap): 8 hashes per lane per key step, not 16
  const bool odd = lo & 1;
  uint64_t dpr[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) dpr[k] = attn_drop_rowpairs(bh * p.T + ib + (odd ? 2 : 0) + k, p.T) + (uint64_t)(lo >> 1);
  const int hsh = odd ? 16 : 0;
  f32x4 oacc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) oacc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint16_t* Pw = Pr + w * (A3K * A3LDT);

  for (int kb = 0; kb < nkb; ++kb) {
    const int j0 = kb * A3K;
    if (kb > 0) {
      __syncthreads();   // every wave is done with the previous step's tiles
      issue(j0);
    }
    __builtin_amdgcn_s_waitcnt(0x70);   // vmcnt(0) lgkmcnt(0): this wave's DMA chunks landed
    __syncthreads();                    // ... and every other wave's
    // ---- scores of this wave's 16 rows x 64 keys: S_ac = Qu K^T, G = Qv Pband^T (fragments read first) ----
    f32x4 ac[4], g[5];
#pragma unroll
    for (int t = 0; t < 4; ++t) ac[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 5; ++t) g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int wb = 48 - 16 * w;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kof = ks * 32 + 8 * q4;
      bf16x8 kf[4], pf[5];
#pragma unroll
      for (int t = 0; t < 4; ++t) kf[t] = *reinterpret_cast<const bf16x8*>(Ks + (16 * t + lo) * LR + kof);
#pragma unroll
      for (int t = 0; t < 5; ++t) pf[t] = *reinterpret_cast<const bf16x8*>(Pr + (wb + 16 * t + lo) * LR + kof);
#pragma unroll
      for (int t = 0; t < 4; ++t) ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fu[ks], kf[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 5; ++t) g[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fv[ks], pf[t], g[t], 0, 0, 0);
    }
    if constexpr (Gm::TAIL) {   // columns 32 KS .. 32 KS + 15: 8-byte fragments, one 16x16x16 MFMA per tile
      const int kof = KS * 32 + 4 * q4;
      bf16x4 kf[4], pf[5];
#pragma unroll
      for (int t = 0; t < 4; ++t) kf[t] = *reinterpret_cast<const bf16x4*>(Ks + (16 * t + lo) * LR + kof);
#pragma unroll
      for (int t = 0; t < 5; ++t) pf[t] = *reinterpret_cast<const bf16x4*>(Pr + (wb + 16 * t + lo) * LR + kof);
#pragma unroll
      for (int t = 0; t < 4; ++t) ac[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fut, kf[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 5; ++t) g[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fvt, pf[t], g[t], 0, 0, 0);
    }
    // raw scores s = S_ac + S_bd (unscaled), the rel_shift by lane permutes
    __syncthreads();   // every wave has read the band tile: its space takes the P^T tiles below
    float s[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float X[5];
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        // (the element is copied out first: __builtin_bit_cast of a vector-element lvalue read element 0 for
        // every r on this compiler -- rows 4q+1..3 of every 16-row tile came out wrong)
        const float gv = g[t][r];
        X[t] = __int_as_float(__builtin_amdgcn_ds_bpermute(bsrc_lane[r], __float_as_int(gv)));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) s[t][r] = ac[t][r] + (bhi[r] ? X[t + 1] : X[t]);
    }
    if (j0 + A3K > lim) {   // the utterance's last key block: keys past its length score -inf
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (j0 + 16 * t + lo >= lim)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[t][r] = -3.0e38f;
    }
    // ---- online softmax (every key block holds a valid key, so the row max is finite after block 0) ----
    float mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
    a3_max16x4(mx[0], mx[1], mx[2], mx[3]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m2[r], mx[r] * sl2);
      const float corr = __builtin_amdgcn_exp2f(m2[r] - mn);
      m2[r] = mn;
      lsum[r] *= corr;
      psum[r] *= corr;
#pragma unroll
      for (int u = 0; u < NU; ++u) oacc[u][r] *= corr;
    }
    float pv[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pv[t][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[t][r], sl2, -m2[r]));
        lsum[r] += pv[t][r];
      }
    if (drop) {
      uint32_t hk[4][2], hp[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int k = 0; k < 2; ++k) hk[t][k] = drop_pair_bits(dkey, dpr[k] + (uint64_t)((j0 >> 1) + 8 * t));
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int k = 0; k < 2; ++k) hp[t][k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)hk[t][k], 0xB1, 0xF, 0xF, false);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t hv = ((r >> 1) == (int)odd) ? hk[t][r & 1] : hp[t][r & 1];
          const bool keep = ((hv >> hsh) & 0xffffu) >= thr;
          pv[t][r] = keep ? pv[t][r] * keep_scale : 0.f;
          psum[r] += pv[t][r];
        }
    }
    // ---- P^T to LDS: key 16 t + lo, rows 4 q4 .. +3 as one 8-byte write; O += Pd V ----
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint2 w2 = make_uint2(pack_bf16x2(pv[t][0], pv[t][1]), pack_bf16x2(pv[t][2], pv[t][3]));
      *reinterpret_cast<uint2*>(Pw + (16 * t + lo) * A3LDT + 4 * q4) = w2;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = a3_tr_frag(Pw, A3LDT, ks * 32, 0, lane);   // A[row lo][key ks 32 + 8 q4 + i]
#pragma unroll
      for (int u = 0; u < NU; ++u)
        oacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, a3_tr_frag(Vs, LR, ks * 32, 16 * u, lane), oacc[u], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();   // Pw is rewritten by the next step
  }
  // ---- per-row log-sum-exp (3e38 for rows without a valid key) and O = centred sum + S_i vc ----
  float lrow[4], prow_sum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    lrow[r] = a3_sum16(lsum[r]);
    prow_sum[r] = drop ? a3_sum16(psum[r]) : 0.f;
  }
  if (p.lse && lo == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r;
      if (i < T) p.lse[bh * p.T + i] = (i < len && lrow[r] > 0.f) ? m2[r] * 0.6931471805599453f + logf(lrow[r]) : 3.0e38f;
    }
  }
  float fin[4], sv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool rv_ok = ib + r < len && lrow[r] > 0.f;
    fin[r] = rv_ok ? 1.f / lrow[r] : 0.f;
    sv[r] = drop ? prow_sum[r] * fin[r] : (rv_ok ? 1.f : 0.f);
  }
  const float* vc = p.cen + bh * 2 * Gm::DKP + Gm::DKP;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int c = 16 * u + lo;
    const float v0 = vc[c];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = ib + r;
      if (i < T && c < dk) p.o[(b * p.T + i) * p.d + hoff + c] = oacc[u][r] * fin[r] + sv[r] * v0;
    }
  }
}

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_attn_kv_prep_elems(int64_t B, int64_t H, int64_t T, int64_t d) {
  if (H <= 0 || d % H) return -1;
  return B * H * kdfm::a3_tp(T) * (kdfm::a3_dkp(d / H) + 8);
}

int64_t kdfm_attn_centre_elems(int64_t B, int64_t H, int64_t d) {
  if (H <= 0 || d % H) return -1;
  return B * H * 2 * kdfm::a3_dkp(d / H);
}

int64_t kdfm_attn_band_prep_elems(int64_t layers, int64_t H, int64_t T, int64_t d) {
  if (H <= 0 || d % H) return -1;
  return layers * H * kdfm::a3_npb(T) * (kdfm::a3_dkp(d / H) + 8);
}

int kdfm_attn_kv_prep(const float* qkv, const int64_t* lengths, uint16_t* kb, uint16_t* vb, float* centre, int64_t B,
                      int64_t H, int64_t T, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(qkv && kb && vb && centre, "null pointer");
  KDFM_REQUIRE(H > 0 && d % H == 0 && d % 4 == 0, "d must be a multiple of H and of 4");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk % 4 == 0 && dk <= 128, "head dim must be a multiple of 4 and <= 128");
  KDFM_REQUIRE(T > 0 && T <= 4096, "T out of range");
  KDFM_REQUIRE((((uintptr_t)qkv | (uintptr_t)kb | (uintptr_t)vb) & 15) == 0, "operands must be 16-byte aligned");
  if (B == 0) return KDFM_OK;
  KDFM_REQUIRE(H <= 64, "at most 64 heads");
  const int64_t Tp = a3_tp(T);
  static const int hpw_env = [] { const char* e = getenv("KDFM_KVPREP_HPW"); return e ? atoi(e) : 0; }();
  // (kind, head) tiles per workgroup: every tile in one workgroup once (Tp / 64) x B fills the chip (the bench's
  // B = 32: 1, 2 or 8 tiles measured the same step time), one tile per workgroup for small batches
  int hpw = hpw_env > 0 ? hpw_env : (Tp / A3K) * B >= 256 ? (int)(2 * H) : 1;
  if (hpw > 2 * H) hpw = (int)(2 * H);
  const dim3 grid((unsigned)(Tp / A3K), (unsigned)B, (unsigned)((2 * H + hpw - 1) / hpw));
  const size_t lds = (size_t)hpw * a3_dkp(dk) * sizeof(float);
  if (a3_dkp(dk) == 128)
    hipLaunchKernelGGL(attn_kv_prep_kernel<128>, grid, dim3(256), lds, as_stream(stream), qkv, lengths, kb, vb, centre, H,
                       (int)T, d, (int)dk, Tp, hpw);
  else if (a3_dkp(dk) == 48)
    hipLaunchKernelGGL(attn_kv_prep_kernel<48>, grid, dim3(256), lds, as_stream(stream), qkv, lengths, kb, vb, centre, H,
                       (int)T, d, (int)dk, Tp, hpw);
  else
    hipLaunchKernelGGL(attn_kv_prep_kernel<64>, grid, dim3(256), lds, as_stream(stream), qkv, lengths, kb, vb, centre, H,
                       (int)T, d, (int)dk, Tp, hpw);
  return check_launch("kdfm_attn_kv_prep");
}

int kdfm_attn_band_prep(const float* pos, int64_t ld_layer, int64_t layers, uint16_t* pb, int64_t H, int64_t T,
                        int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(pos && pb, "null pointer");
  KDFM_REQUIRE(H > 0 && d % H == 0 && d % 4 == 0, "d must be a multiple of H and of 4");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk % 4 == 0 && dk <= 128, "head dim must be a multiple of 4 and <= 128");
  KDFM_REQUIRE(T > 0 && T <= 4096 && layers > 0, "T / layers out of range");
  KDFM_REQUIRE(layers == 1 || ld_layer >= (2 * T - 1) * d, "layer stride too small");
  KDFM_REQUIRE((((uintptr_t)pos | (uintptr_t)pb) & 15) == 0 && ld_layer % 4 == 0, "operands must be 16-byte aligned");
  const int64_t npb = a3_npb(T);
  const dim3 grid((unsigned)ceil_div(npb, 64), (unsigned)(layers * H));
  if (a3_dkp(dk) == 128)
    hipLaunchKernelGGL(attn_band_prep_kernel<128>, grid, dim3(256), 0, as_stream(stream), pos, ld_layer, pb, H, 2 * T - 1, d,
                       (int)dk, npb);
  else if (a3_dkp(dk) == 48)
    hipLaunchKernelGGL(attn_band_prep_kernel<48>, grid, dim3(256), 0, as_stream(stream), pos, ld_layer, pb, H, 2 * T - 1, d,
                       (int)dk, npb);
  else
    hipLaunchKernelGGL(attn_band_prep_kernel<64>, grid, dim3(256), 0, as_stream(stream), pos, ld_layer, pb, H, 2 * T - 1, d,
                       (int)dk, npb);
  return check_launch("kdfm_attn_band_prep");
}

int kdfm_relpos_attn_fwd3(const float* qu, const float* qv, const uint16_t* kb, const uint16_t* vb, const float* centre,
                          const uint16_t* pb, const int64_t* lengths, float* o, float* lse, int64_t B, int64_t H,
                          int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                          void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(qu && qv && kb && vb && centre && pb && o, "null pointer");
  KDFM_REQUIRE(H > 0 && d % H == 0 && d % 4 == 0, "d must be a multiple of H and of 4");
  const int64_t dk = d / H;
  KDFM_REQUIRE(dk % 4 == 0 && dk <= 128, "head dim must be a multiple of 4 and <= 128");
  KDFM_REQUIRE(T > 0 && T <= 4096, "T out of range");
  KDFM_REQUIRE(dropout_p == 0.f || seed, "dropout needs a seed");
  KDFM_REQUIRE((((uintptr_t)qu | (uintptr_t)qv | (uintptr_t)kb | (uintptr_t)vb | (uintptr_t)pb) & 15) == 0,
               "operands must be 16-byte aligned");
  if (B == 0) return KDFM_OK;
  Attn3P p;
  p.qu = qu; p.qv = qv; p.kb = kb; p.vb = vb; p.cen = centre; p.pb = pb; p.lens = lengths;
  p.o = o; p.lse = lse;
  p.B = B; p.H = H; p.T = T; p.d = d; p.dk = dk; p.Tp = a3_tp(T); p.npb = a3_npb(T);
  p.scale = scale; p.p_drop = dropout_p; p.seed = seed; p.rng_stream = rng_stream;
  const dim3 grid((unsigned)ceil_div(T, A3Q), (unsigned)(B * H));
  hipStream_t st = as_stream(stream);
  if (dk > 64)
    hipLaunchKernelGGL(relpos_attn_fwd3_kernel<8>, grid, dim3(256), 0, st, p);
  else if (dk > 48)
    hipLaunchKernelGGL(relpos_attn_fwd3_kernel<4>, grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(relpos_attn_fwd3_kernel<3>, grid, dim3(256), 0, st, p);
  return check_launch("kdfm_relpos_attn_fwd3");
}

}  // extern "C"
