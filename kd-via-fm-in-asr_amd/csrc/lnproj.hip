// LayerNorm-fused input projections of the Conformer attention and convolution modules, forward and
// data-gradient/LayerNorm backward (bf16 MFMA, f32 state; building blocks in lnblock.h).
//
// Reference: ConformerLayer.forward (built conformer_encoder.py:450-472,
// called :685-692):
//   QKV:  ln = LN_att(r);  q|k|v = ln W_qkv^T + b;  qu = q + pos_bias_u, qv = q + pos_bias_v
//         (RelPositionMultiHeadAttention's linear_q/k/v and the two positional biases)
//   GLU:  ln = LN_conv(r); a|gate = ln W_pw1^T + b;  g = a * sigmoid(gate), zero on padded frames
//         (ConformerConvolution's pointwise_conv1 + GLU + the pad mask before the depthwise conv)
// The unfused path ran LN, the projection GEMM and the prep / GLU kernels as separate launches with
// the LN output and the projection in HBM; here a wave holds LN(r) of its 32 rows as bf16 MFMA
// operands in registers and emits the projection's consumers directly.  Training saves the row
// statistics and the bf16 LN output (the weight-gradient operand; exactly the values the GEMM path
// rounds at MFMA staging).  The backward kernels take the projection's output gradient, form
// dln = W^T dproj through MFMAs (GLU: the projection is recomputed from LN(r) for GLU'), write the bf16
// dproj (dW = dproj^T ln on the row-parallel wgrad kernel) and finish the LayerNorm backward + residual.
//
// Work split: 3 waves per 32-row tile (one per q / k / v kind, or one per 32-feature GLU group),
// 2 tiles per workgroup (384 threads); backward partial dln sums are added in wave order through LDS.
#include "lnblock.h"
#include "wimg.h"

namespace kdfm {
namespace {

using namespace lnb;

constexpr int LP_NP = 3;                   // waves per 32-row tile
constexpr int LP_NT = 2 * LP_NP * 64;      // 384 threads = 2 row tiles
constexpr int LP_ROWS = 64;
enum { LP_QKV = 0, LP_GLU = 1 };

template <int MODE> struct Kinds { static constexpr int G = MODE == LP_QKV ? 3 : 2; };

// Forward image, unit-major.  QKV unit u = 3 t + g (feature tile t of kind g = q/k/v), KS1 fragments;
// GLU unit u = t, 2 KS1 fragments [a tile | gate tile].  Fragment (g, t, ks), lane (r, h), j < 8:
//   W[g d + 32 t + r][16 ks + 8 h + j]
// Backward image, one block per feature group t: W^T fragments (g, s2, mt) at (2 g + s2) DT + mt:
//   W[g d + 32 t + 16 s2 + 8 h + j][32 mt + r]     (A of dln^T = W^T dproj^T)
// preceded, for GLU, by the forward unit t (the backward recomputes a | gate).
template <int KS1, int DT, int MODE>
struct LpGeo {
  static constexpr int G = Kinds<MODE>::G;
  static constexpr int UF = MODE == LP_QKV ? KS1 : 2 * KS1;       // fragments per forward unit
  static constexpr int NU = MODE == LP_QKV ? 3 * DT : DT;          // forward units
  static constexpr int TB = 2 * G * DT;                            // W^T fragments per group
  static constexpr int BB = (MODE == LP_GLU ? 2 * KS1 : 0) + TB;   // backward block
};

__global__ __launch_bounds__(256) void lnproj_wprep_kernel(const float* __restrict__ W, uint16_t* __restrict__ img,
                                                           int d, int KS1, int DT, int mode, int bwd, int64_t total) {
  const int64_t gidx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gidx >= total) return;
  const int lane = (int)(gidx & 63);
  const int f = (int)(gidx >> 6);
  float v[8];
  wimg::lnproj_frag(W, d, KS1, DT, mode, bwd, f, lane, v);
  *reinterpret_cast<bf16x8*>(img + ((int64_t)f * 64 + lane) * 8) = pack_bf16x8<bf16x8>(v);
}

struct LpFwd {
  const float* x; const float* g; const float* b; float eps;
  const uint16_t* img; const float* bias;
  const float* pu; const float* pv; float* qu; float* qv; float* qkv;   // QKV
  float* gout; const int64_t* lens; int64_t T;                          // GLU
  float* mean; float* rstd; uint16_t* ln_h;
  int64_t rows; int d;
};

template <int KS1, int DT, int MODE>
__global__ __launch_bounds__(LP_NT) void lnproj_fwd_kernel(LpFwd a) {
  using Gm = LpGeo<KS1, DT, MODE>;
  using St = DmaStager<Gm::UF, 0, Gm::UF, LP_NP, LP_NT>;
  extern __shared__ __attribute__((aligned(16))) uint4 lp_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, p = wave % LP_NP, tile = wave / LP_NP;
  const int64_t row = (int64_t)blockIdx.x * LP_ROWS + tile * 32 + (lane & 31);
  const bool ok = row < a.rows;
  const int d = a.d;
  const uint4* img = reinterpret_cast<const uint4*>(a.img);
  St::issue(img, 0, Gm::NU, lp_lds, 0);
  float xv[KS1][8];
  ln_load<KS1>(a.x, row, ok, d, h, xv);
  bool live = ok;
  if (MODE == LP_GLU && ok && a.lens) live = (row % a.T) < a.lens[row / a.T];
  constexpr int S = (Gm::NU + LP_NP - 1) / LP_NP;
  // projection bias (and the positional biases) in LDS: a global load inside the loop would wait
  // (in-order vmcnt) for the next stage's prefetch
  float* vec_s = reinterpret_cast<float*>(lp_lds + (S > 1 ? 2 : 1) * St::UNITS);
  // [bias | pos_bias_u | pos_bias_v | gamma | beta] (QKV) or [bias | gamma | beta] (GLU), filled while the
  // row loads and the stage-0 DMA are in flight; the LayerNorm runs after the barrier
  const int ng = (MODE == LP_QKV ? 5 : 2) * d;
  if (MODE == LP_QKV)
    fill_vec5<7 * 32 * DT, LP_NT>(vec_s, a.bias, 3 * d, a.pu, d, a.pv, d, a.g, d, a.b, d);
  else
    fill_vec5<4 * 32 * DT, LP_NT>(vec_s, a.bias, 2 * d, a.g, d, a.b, d, a.b, 0, a.b, 0);
  __syncthreads();
  float mean = 0.f, rstd = 0.f;
  bf16x8 bx[KS1];
  ln_finish<KS1>(xv, vec_s + ng, vec_s + ng + d, row, ok, d, h, a.eps, false, mean, rstd, bx,
                 p == 0 ? a.ln_h : nullptr);
  if (a.mean && p == 0 && h == 0 && ok) {
    a.mean[row] = mean;
    a.rstd[row] = rstd;
  }
  // the outputs leave as buffer stores every lane issues, a fixed count per unit (QKV: 8 -- the k / v
  // waves add 4 range-dropped ones; GLU: 4), so the stage barrier counts past them (dma_barrier)
  static_assert(Gm::NU % LP_NP == 0, "every wave has a unit in every stage");
  constexpr uint32_t OOB = 0x80000000u;
  constexpr int NST = MODE == LP_QKV ? 8 : 4;
  const int rd4 = (int)(a.rows * d * 4);
  const __amdgpu_buffer_rsrc_t r_a = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(MODE == LP_QKV ? a.qu : a.gout), (short)0, rd4, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_b = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(MODE == LP_QKV ? a.qv : a.gout), (short)0, rd4, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_k = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(MODE == LP_QKV ? a.qkv : a.gout), (short)0, MODE == LP_QKV ? 3 * rd4 : rd4, 0x00020000);
  for (int s = 0; s < S; ++s) {
    const int u = s * LP_NP + p;
    // this unit's bias vectors are read from LDS before the next stage's DMA is issued (an LDS read
    // while an LDS-DMA is in flight makes the compiler drain it first)
    float4 vb[2][4], vq[2][4];
    {
      const int uu = u < Gm::NU ? u : 0;
      const int t = MODE == LP_QKV ? uu / 3 : uu, g = MODE == LP_QKV ? uu % 3 : 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = 32 * t + 8 * q + 4 * h < d ? 32 * t + 8 * q + 4 * h : 0;
        vb[0][q] = *reinterpret_cast<const float4*>(vec_s + g * d + n0);
        vb[1][q] = *reinterpret_cast<const float4*>(vec_s + d + n0);   // GLU: gate bias
        vq[0][q] = *reinterpret_cast<const float4*>(vec_s + 3 * (MODE == LP_QKV) * d + n0);
        vq[1][q] = *reinterpret_cast<const float4*>(vec_s + 4 * (MODE == LP_QKV) * d + n0);
      }
    }
    if (s + 1 < S) St::issue(img, s + 1, Gm::NU, lp_lds, (s + 1) & 1);
    if (u < Gm::NU) {
      const uint4* W = St::block(lp_lds, s & 1, p);
      if constexpr (MODE == LP_QKV) {
        const int t = u / 3, g = u % 3;
        f32x16 acc = zero16();
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) acc = mfma32(W[ks * FRAG_U4 + lane], bx[ks], acc);
        const __amdgpu_buffer_rsrc_t r1 = g == 0 ? r_a : r_k;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n0 = 32 * t + 8 * q + 4 * h;
          const bool in = ok && n0 < d;
          const float4 bb = vb[0][q];
          const float v0 = acc[4 * q] + bb.x, v1 = acc[4 * q + 1] + bb.y, v2 = acc[4 * q + 2] + bb.z,
                      v3 = acc[4 * q + 3] + bb.w;
          const float4 uu = vq[0][q], vv = vq[1][q];
          // qu (g == 0) or the k / v slice of qkv; then qv (g == 0) or a dropped store
          const f32x4 o1 = g == 0 ? f32x4{v0 + uu.x, v1 + uu.y, v2 + uu.z, v3 + uu.w} : f32x4{v0, v1, v2, v3};
          const f32x4 o2 = f32x4{v0 + vv.x, v1 + vv.y, v2 + vv.z, v3 + vv.w};
          const uint32_t off1 = !in ? OOB : (uint32_t)((g == 0 ? row * d + n0 : row * 3 * d + g * d + n0) * 4);
          const uint32_t off2 = (!in || g != 0) ? OOB : (uint32_t)((row * d + n0) * 4);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, o1), r1, off1, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, o2), r_b, off2, 0, 0);
        }
      } else {
        const int t = u;
        f32x16 aa = zero16(), ag = zero16();
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
          aa = mfma32(W[ks * FRAG_U4 + lane], bx[ks], aa);
          ag = mfma32(W[(KS1 + ks) * FRAG_U4 + lane], bx[ks], ag);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n0 = 32 * t + 8 * q + 4 * h;
          const bool in = ok && n0 < d;
          const float4 ba = vb[0][q];
          const float4 bg = vb[1][q];
          const float va[4] = {aa[4 * q] + ba.x, aa[4 * q + 1] + ba.y, aa[4 * q + 2] + ba.z, aa[4 * q + 3] + ba.w};
          const float vg[4] = {ag[4 * q] + bg.x, ag[4 * q + 1] + bg.y, ag[4 * q + 2] + bg.z, ag[4 * q + 3] + bg.w};
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = live ? va[i] * sigmoidf_(vg[i]) : 0.f;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, f32x4{o[0], o[1], o[2], o[3]}), r_a,
                                                 in ? (uint32_t)((row * d + n0) * 4) : OOB, 0, 0);
        }
      }
    }
    dma_barrier<NST>();   // stage s + 1 landed; this unit's NST output stores stay in flight
  }
}

struct LpBwd {
  const float* dqu; const float* dqv; const float* dqkv; uint16_t* dproj_h;   // QKV
  const float* dg; const int64_t* lens; int64_t T; const float* bias;        // GLU
  const float* x; const float* mean; const float* rstd; const float* g; const float* b;
  const uint16_t* img; const float* dres; float* dx; uint16_t* ln_h; float* part;
  int64_t rows, nparts; int d;
  float* part_uv;   // QKV: optional pos_bias_u / pos_bias_v column-sum partials
};

// dln partials of the 3 waves of a tile -> wave 0 (fixed order 0 + 1 + 2), then the LN backward
template <int DT>
__device__ __forceinline__ void lp_finish(f32x16 (&acc)[DT], float* red, const LpBwd& a, int p, int tile, int lane,
                                          int64_t row, bool ok, float mean, float rstd) {
  float* rt = red + tile * (LP_NP - 1) * (DT * 16 * 64);
  if (p > 0) {
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) rt[((p - 1) * DT * 16 + mt * 16 + e) * 64 + lane] = acc[mt][e];
  }
  __syncthreads();
  if (p > 0) return;
  float dl[DT * 16];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float v = acc[mt][e];
#pragma unroll
      for (int w = 0; w < LP_NP - 1; ++w) v += rt[(w * DT * 16 + mt * 16 + e) * 64 + lane];
      dl[mt * 16 + e] = v;
    }
  ln_backward_rows<DT>(dl, a.x, a.g, a.dres, a.dx, a.part, a.nparts, row - (lane & 31), row, ok, a.d, mean, rstd,
                       lane);
}

template <int KS1, int DT>
__global__ __launch_bounds__(LP_NT) void ln_qkv_bwd_kernel(LpBwd a) {
  using Gm = LpGeo<KS1, DT, LP_QKV>;
  using St = DmaStager<Gm::TB, 0, Gm::TB, 1, LP_NT>;
  extern __shared__ __attribute__((aligned(16))) uint4 lp_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, p = wave % LP_NP, tile = wave / LP_NP;   // p = kind (q, k, v)
  const int64_t row = (int64_t)blockIdx.x * LP_ROWS + tile * 32 + (lane & 31);
  const bool ok = row < a.rows;
  const int d = a.d;
  const uint4* img = reinterpret_cast<const uint4*>(a.img);
  St::issue(img, 0, DT, lp_lds, 0);
  // every prologue load first (the dproj rows, row statistics, x rows of the q wave), masks by multiply,
  // then the bf16 stores: a load issued after a store, or a select on a loaded value, is waited for
  // one at a time
  // B operands of this kind: dproj features 32 t + 16 s2 + 8 h .. +7
  float4 r0[2 * DT], r1[2 * DT];
#pragma unroll
  for (int k = 0; k < 2 * DT; ++k) {
    const int f0 = 16 * k + 8 * h;
    const bool in = ok && f0 < d;
    const float* src = p == 0 ? a.dqu + (in ? row * d + f0 : 0) : a.dqkv + (in ? row * 3 * d + p * d + f0 : 0);
    r0[k] = reinterpret_cast<const float4*>(src)[0];
    r1[k] = reinterpret_cast<const float4*>(src)[1];
  }
  float4 w0[2 * DT], w1[2 * DT];
  if (p == 0) {
#pragma unroll
    for (int k = 0; k < 2 * DT; ++k) {
      const int f0 = 16 * k + 8 * h;
      const bool in = ok && f0 < d;
      w0[k] = reinterpret_cast<const float4*>(a.dqv + (in ? row * d + f0 : 0))[0];
      w1[k] = reinterpret_cast<const float4*>(a.dqv + (in ? row * d + f0 : 0))[1];
    }
  }
  const int64_t rc = ok ? row : 0;
  const float rm = ok ? 1.f : 0.f;
  float mean = a.mean[rc] * rm, rstd = a.rstd[rc] * rm;
  float xv[KS1][8];
  if (p == 0) ln_load<KS1>(a.x, row, ok, d, h, xv);
  bf16x8 bop[2 * DT];
#pragma unroll
  for (int k = 0; k < 2 * DT; ++k) {
    const int f0 = 16 * k + 8 * h;
    const float m = (ok && f0 < d) ? 1.f : 0.f;
    float v[8] = {r0[k].x, r0[k].y, r0[k].z, r0[k].w, r1[k].x, r1[k].y, r1[k].z, r1[k].w};
    if (p == 0) {
      v[0] += w0[k].x; v[1] += w0[k].y; v[2] += w0[k].z; v[3] += w0[k].w;
      v[4] += w1[k].x; v[5] += w1[k].y; v[6] += w1[k].z; v[7] += w1[k].w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= m;
    bop[k] = pack_bf16x8<bf16x8>(v);
  }
#pragma unroll
  for (int k = 0; k < 2 * DT; ++k) {
    const int f0 = 16 * k + 8 * h;
    if (ok && f0 < d) *reinterpret_cast<bf16x8*>(a.dproj_h + row * 3 * d + p * d + f0) = bop[k];
  }
  if (p == 0) {   // bf16 LN output: the weight-gradient operand
    bf16x8 bx[KS1];
    ln_finish<KS1>(xv, a.g, a.b, row, ok, d, h, 0.f, true, mean, rstd, bx, a.ln_h);
  }
  f32x16 acc[DT];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt) acc[mt] = zero16();
  __syncthreads();
  for (int t = 0; t < DT; ++t) {
    if (t + 1 < DT) St::issue(img, t + 1, DT, lp_lds, (t + 1) & 1);
    const uint4* W = St::block(lp_lds, t & 1, 0);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int mt = 0; mt < DT; ++mt)
        acc[mt] = mfma32(W[((2 * p + s2) * DT + mt) * FRAG_U4 + lane], bop[2 * t + s2], acc[mt]);
    __syncthreads();
  }
  if (a.part_uv && p > 0) {
    // pos_bias_u / pos_bias_v gradients (column sums of dqu / dqv) as 16-row-group partials in the
    // LayerNorm partial layout (part_uv[grp][2d]), folded by the layer's kdfm_ln_fold with its LNs
    constexpr int NV = 2 * DT * 8;
    const float* src = p == 1 ? a.dqu : a.dqv;
    float v0[NV];
#pragma unroll
    for (int k = 0; k < 2 * DT; ++k) {
      const int f0 = 16 * k + 8 * h;
      const bool in = ok && f0 < d;
      const float4* q = reinterpret_cast<const float4*>(src + (in ? row * d + f0 : 0));
      const float4 u0 = q[0], u1 = q[1];
      const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) v0[8 * k + j] = in ? u[j] : 0.f;
    }
    float r1[NV / 2], r2[NV / 4], r3[NV / 8], r4[NV / 16];
    rs_step<NV, 8>(v0, r1, lane);
    rs_step<NV / 2, 4>(r1, r2, lane);
    rs_step<NV / 4, 2>(r2, r3, lane);
    rs_step<NV / 8, 1>(r3, r4, lane);
    const int64_t grp = (row - (lane & 31)) / 16 + ((lane >> 4) & 1);
    const int base = ((lane & 8) ? NV / 2 : 0) + ((lane & 4) ? NV / 4 : 0) + ((lane & 2) ? NV / 8 : 0) +
                     ((lane & 1) ? NV / 16 : 0);
    if (grp < a.nparts) {
#pragma unroll
      for (int j = 0; j < NV / 16; ++j) {
        const int e = base + j;
        const int f = 16 * (e / 8) + 8 * h + (e % 8);
        if (f < d) a.part_uv[grp * 2 * d + (p - 1) * d + f] = r4[j];
      }
    }
  }
  lp_finish<DT>(acc, reinterpret_cast<float*>(lp_lds), a, p, tile, lane, row, ok, mean, rstd);
}

template <int KS1, int DT>
__global__ __launch_bounds__(LP_NT) void ln_glu_bwd_kernel(LpBwd a) {
  using Gm = LpGeo<KS1, DT, LP_GLU>;
  using St = DmaStager<Gm::BB, 0, Gm::BB, LP_NP, LP_NT>;
  static_assert(DT <= LP_NP, "one GLU group per wave");
  extern __shared__ __attribute__((aligned(16))) uint4 lp_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, p = wave % LP_NP, tile = wave / LP_NP;   // p = GLU feature group
  const int64_t row = (int64_t)blockIdx.x * LP_ROWS + tile * 32 + (lane & 31);
  const bool ok = row < a.rows;
  const int d = a.d;
  St::issue(reinterpret_cast<const uint4*>(a.img), 0, DT, lp_lds, 0);
  // every prologue load first (row statistics, x rows, this group's biases and dg rows, the length),
  // then the LayerNorm and its bf16 store: a load issued after a store is waited for one at a time
  const int64_t rc = ok ? row : 0;
  const float rm = ok ? 1.f : 0.f;
  float mean = a.mean[rc] * rm, rstd = a.rstd[rc] * rm;
  float xv[KS1][8];
  ln_load<KS1>(a.x, row, ok, d, h, xv);
  const int t = p;
  float4 bav[4], bgv[4], dgr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 32 * t + 8 * q + 4 * h;
    const bool in = ok && n0 < d;
    bav[q] = *reinterpret_cast<const float4*>(a.bias + (n0 < d ? n0 : 0));
    bgv[q] = *reinterpret_cast<const float4*>(a.bias + d + (n0 < d ? n0 : 0));
    dgr[q] = *reinterpret_cast<const float4*>(a.dg + (in ? row * d + n0 : 0));
  }
  const int64_t ln = a.lens ? a.lens[rc / a.T] : a.T;
  const bool live = ok && (row % a.T) < ln;
  bf16x8 bx[KS1];
  ln_finish<KS1>(xv, a.g, a.b, row, ok, d, h, 0.f, true, mean, rstd, bx, p == 0 ? a.ln_h : nullptr);
  f32x16 acc[DT];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt) acc[mt] = zero16();
  __syncthreads();
  if (t < DT) {
    const uint4* W = St::block(lp_lds, 0, p);
    f32x16 aa = zero16(), ag = zero16();
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      aa = mfma32(W[ks * FRAG_U4 + lane], bx[ks], aa);
      ag = mfma32(W[(KS1 + ks) * FRAG_U4 + lane], bx[ks], ag);
    }
    uint32_t pa[4][2], pg[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = 32 * t + 8 * q + 4 * h;
      const bool in = live && n0 < d;
      const float4 ba = bav[q], bg = bgv[q], dgv = dgr[q];
      const float va[4] = {aa[4 * q] + ba.x, aa[4 * q + 1] + ba.y, aa[4 * q + 2] + ba.z, aa[4 * q + 3] + ba.w};
      const float vg[4] = {ag[4 * q] + bg.x, ag[4 * q + 1] + bg.y, ag[4 * q + 2] + bg.z, ag[4 * q + 3] + bg.w};
      const float gv[4] = {dgv.x, dgv.y, dgv.z, dgv.w};
      float da[4], dgt[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float s = sigmoidf_(vg[i]);
        da[i] = in ? gv[i] * s : 0.f;
        dgt[i] = in ? gv[i] * va[i] * s * (1.f - s) : 0.f;
      }
      pack4(pa[q], da);
      pack4(pg[q], dgt);
    }
    bf16x8 ba2[2], bg2[2];
    tile_operands(pa, ba2);
    tile_operands(pg, bg2);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int f0 = 32 * t + 16 * s2 + 8 * h;
      if (ok && f0 < d) {
        *reinterpret_cast<bf16x8*>(a.dproj_h + row * 2 * d + f0) = ba2[s2];
        *reinterpret_cast<bf16x8*>(a.dproj_h + row * 2 * d + d + f0) = bg2[s2];
      }
#pragma unroll
      for (int mt = 0; mt < DT; ++mt) {
        acc[mt] = mfma32(W[(2 * KS1 + (0 + s2) * DT + mt) * FRAG_U4 + lane], ba2[s2], acc[mt]);
        acc[mt] = mfma32(W[(2 * KS1 + (2 + s2) * DT + mt) * FRAG_U4 + lane], bg2[s2], acc[mt]);
      }
    }
  }
  __syncthreads();   // every wave is done with the staged image before the reduction reuses the LDS
  lp_finish<DT>(acc, reinterpret_cast<float*>(lp_lds), a, p, tile, lane, row, ok, mean, rstd);
}

template <typename K>
void lp_allow_lds(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int KS1, int DT, int MODE>
int launch_lp_fwd(const LpFwd& a, hipStream_t st) {
  using Gm = LpGeo<KS1, DT, MODE>;
  static bool once = (lp_allow_lds(lnproj_fwd_kernel<KS1, DT, MODE>), true);
  (void)once;
  constexpr int S = (Gm::NU + LP_NP - 1) / LP_NP;
  const size_t lds = (size_t)(S > 1 ? 2 : 1) * LP_NP * Gm::UF * 1024 + (size_t)(MODE == LP_QKV ? 7 : 4) * a.d * 4;
  hipLaunchKernelGGL((lnproj_fwd_kernel<KS1, DT, MODE>), dim3((unsigned)ceil_div(a.rows, LP_ROWS)), dim3(LP_NT), lds, st,
                     a);
  return check_launch(MODE == LP_QKV ? "kdfm_ln_qkv_fwd" : "kdfm_ln_glu_fwd");
}

constexpr size_t lp_red_bytes(int DT) { return (size_t)2 * (LP_NP - 1) * DT * 16 * 64 * 4; }

template <int KS1, int DT>
int launch_qkv_bwd(const LpBwd& a, hipStream_t st) {
  using Gm = LpGeo<KS1, DT, LP_QKV>;
  static bool once = (lp_allow_lds(ln_qkv_bwd_kernel<KS1, DT>), true);
  (void)once;
  const size_t stage = (size_t)2 * Gm::TB * 1024;
  const size_t lds = stage > lp_red_bytes(DT) ? stage : lp_red_bytes(DT);
  hipLaunchKernelGGL((ln_qkv_bwd_kernel<KS1, DT>), dim3((unsigned)ceil_div(a.rows, LP_ROWS)), dim3(LP_NT), lds, st, a);
  return check_launch("kdfm_ln_qkv_bwd");
}

template <int KS1, int DT>
int launch_glu_bwd(const LpBwd& a, hipStream_t st) {
  using Gm = LpGeo<KS1, DT, LP_GLU>;
  static bool once = (lp_allow_lds(ln_glu_bwd_kernel<KS1, DT>), true);
  (void)once;
  const size_t stage = (size_t)LP_NP * Gm::BB * 1024;
  const size_t lds = stage > lp_red_bytes(DT) ? stage : lp_red_bytes(DT);
  hipLaunchKernelGGL((ln_glu_bwd_kernel<KS1, DT>), dim3((unsigned)ceil_div(a.rows, LP_ROWS)), dim3(LP_NT), lds, st, a);
  return check_launch("kdfm_ln_glu_bwd");
}

int64_t lp_img_frags(int mode, int64_t d, int bwd) {
  int KS1, DT;
  if (ln_dims(d, KS1, DT) != 0 || (mode != LP_QKV && mode != LP_GLU)) return -1;
  if (bwd && DT != 3) return -1;   // backward variants compiled for d in (80, 96]
  const int G = mode == LP_QKV ? 3 : 2;
  if (!bwd) return (int64_t)(mode == LP_QKV ? 3 * DT * KS1 : DT * 2 * KS1);
  return (int64_t)DT * ((mode == LP_GLU ? 2 * KS1 : 0) + 2 * G * DT);
}

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_lnproj_img_elems(int32_t kind, int64_t d, int32_t bwd) {
  const int64_t f = kdfm::lp_img_frags(kind, d, bwd);
  return f < 0 ? 0 : f * 512;
}

int kdfm_lnproj_wprep(int32_t kind, const float* W, uint16_t* img, int64_t d, int32_t bwd, void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(W && img, "null pointer");
  const int64_t f = lp_img_frags(kind, d, bwd);
  KDFM_REQUIRE(f > 0, "unsupported (kind, d, direction)");
  KDFM_REQUIRE(al16(img), "img must be 16-byte aligned");
  int KS1, DT;
  ln_dims(d, KS1, DT);
  const int64_t total = f * 64;
  hipLaunchKernelGGL(lnproj_wprep_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, as_stream(stream), W,
                     img, (int)d, KS1, DT, (int)kind, (int)bwd, total);
  return check_launch("kdfm_lnproj_wprep");
}

int kdfm_ln_qkv_fwd(const float* x, const float* ln_g, const float* ln_b, float ln_eps, const uint16_t* img,
                    const float* bias, const float* pos_u, const float* pos_v, float* qu, float* qv, float* qkv,
                    float* mean, float* rstd, uint16_t* ln_h, int64_t rows, int64_t d, void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(x && ln_g && ln_b && img && bias && pos_u && pos_v && qu && qv && qkv, "null pointer");
  KDFM_REQUIRE((mean == nullptr) == (rstd == nullptr), "mean and rstd go together");
  int KS1, DT;
  KDFM_REQUIRE(ln_dims(d, KS1, DT) == 0, "unsupported d");
  KDFM_REQUIRE(rows * 3 * d * 4 <= (int64_t)INT32_MAX - 64, "rows x 3d exceeds the 2 GB buffer-store range");
  KDFM_REQUIRE(al16(x) && al16(ln_g) && al16(ln_b) && al16(img) && al16(bias) && al16(pos_u) && al16(pos_v) &&
                   al16(qu) && al16(qv) && al16(qkv) && al16(ln_h),
               "operands must be 16-byte aligned");
  if (rows <= 0) return KDFM_OK;
  LpFwd a{x, ln_g, ln_b, ln_eps, img, bias, pos_u, pos_v, qu, qv, qkv, nullptr, nullptr, 1, mean, rstd, ln_h,
          rows, (int)d};
  hipStream_t st = as_stream(stream);
  if (KS1 == 6) return launch_lp_fwd<6, 3, LP_QKV>(a, st);
  if (KS1 == 11) return launch_lp_fwd<11, 6, LP_QKV>(a, st);
  return launch_lp_fwd<12, 6, LP_QKV>(a, st);
}

int kdfm_ln_glu_fwd(const float* x, const float* ln_g, const float* ln_b, float ln_eps, const uint16_t* img,
                    const float* bias, const int64_t* lengths, int64_t T, float* g, float* mean, float* rstd,
                    uint16_t* ln_h, int64_t rows, int64_t d, void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(x && ln_g && ln_b && img && bias && g, "null pointer");
  KDFM_REQUIRE((mean == nullptr) == (rstd == nullptr), "mean and rstd go together");
  KDFM_REQUIRE(T > 0 && rows % T == 0, "rows must be whole utterances of T frames");
  int KS1, DT;
  KDFM_REQUIRE(ln_dims(d, KS1, DT) == 0, "unsupported d");
  KDFM_REQUIRE(rows * d * 4 <= (int64_t)INT32_MAX - 64, "rows x d exceeds the 2 GB buffer-store range");
  KDFM_REQUIRE(al16(x) && al16(ln_g) && al16(ln_b) && al16(img) && al16(bias) && al16(g) && al16(ln_h),
               "operands must be 16-byte aligned");
  if (rows <= 0) return KDFM_OK;
  LpFwd a{x, ln_g, ln_b, ln_eps, img, bias, nullptr, nullptr, nullptr, nullptr, nullptr, g, lengths, T, mean, rstd,
          ln_h, rows, (int)d};
  hipStream_t st = as_stream(stream);
  if (KS1 == 6) return launch_lp_fwd<6, 3, LP_GLU>(a, st);
  if (KS1 == 11) return launch_lp_fwd<11, 6, LP_GLU>(a, st);
  return launch_lp_fwd<12, 6, LP_GLU>(a, st);
}

int kdfm_ln_qkv_bwd(const float* dqu, const float* dqv, const float* dqkv, const float* x, const float* mean,
                    const float* rstd, const float* ln_g, const float* ln_b, const uint16_t* img, const float* dres,
                    float* dx, uint16_t* ln_h, uint16_t* dqkv_h, float* part, float* part_uv, int64_t rows, int64_t d,
                    void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(dqu && dqv && dqkv && x && mean && rstd && ln_g && ln_b && img && dres && dx && ln_h && dqkv_h && part,
               "null pointer");
  KDFM_REQUIRE(lp_img_frags(LP_QKV, d, 1) > 0, "unsupported d (backward: d in (80, 96])");
  KDFM_REQUIRE(al16(dqu) && al16(dqv) && al16(dqkv) && al16(x) && al16(ln_g) && al16(ln_b) && al16(img) && al16(dres) &&
                   al16(dx) && al16(ln_h) && al16(dqkv_h),
               "operands must be 16-byte aligned");
  if (rows <= 0) return KDFM_OK;
  LpBwd a{dqu, dqv, dqkv, dqkv_h, nullptr, nullptr, 1, nullptr, x, mean, rstd, ln_g, ln_b, img, dres, dx, ln_h, part,
          rows, ceil_div(rows, 16), (int)d, part_uv};
  return launch_qkv_bwd<6, 3>(a, as_stream(stream));
}

int kdfm_ln_glu_bwd(const float* dg, const float* x, const float* mean, const float* rstd, const float* ln_g,
                    const float* ln_b, const uint16_t* img, const float* bias, const int64_t* lengths, int64_t T,
                    const float* dres, float* dx, uint16_t* ln_h, uint16_t* da_h, float* part, int64_t rows,
                    int64_t d, void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(dg && x && mean && rstd && ln_g && ln_b && img && bias && dres && dx && ln_h && da_h && part,
               "null pointer");
  KDFM_REQUIRE(T > 0 && rows % T == 0, "rows must be whole utterances of T frames");
  KDFM_REQUIRE(lp_img_frags(LP_GLU, d, 1) > 0, "unsupported d (backward: d in (80, 96])");
  KDFM_REQUIRE(al16(dg) && al16(x) && al16(ln_g) && al16(ln_b) && al16(img) && al16(bias) && al16(dres) && al16(dx) &&
                   al16(ln_h) && al16(da_h),
               "operands must be 16-byte aligned");
  if (rows <= 0) return KDFM_OK;
  LpBwd a{nullptr, nullptr, nullptr, da_h, dg, lengths, T, bias, x, mean, rstd, ln_g, ln_b, img, dres, dx, ln_h, part,
          rows, ceil_div(rows, 16), (int)d, nullptr};
  return launch_glu_bwd<6, 3>(a, as_stream(stream));
}

}  // extern "C"
