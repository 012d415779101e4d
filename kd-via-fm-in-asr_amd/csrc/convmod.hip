// Conformer convolution module pieces (NeMo ConformerConvolution, Appendix A.8; built at
// conformer_encoder.py:450-472 with conv_kernel_size 31, conv_norm_type batch_norm):
//   GLU(dim=channels) + pad-mask  ->  depthwise Conv1d(k=31, pad 15/15)  ->  BatchNorm1d
//   (batch statistics in training, running statistics in eval)  ->  SiLU.
// Layout: channels-last rows (B*T, C).  The depthwise conv stages a (64+k-1) x 64 frame x channel
// tile in LDS (coalesced along channels) so each input element is read from HBM once per tile.
// BatchNorm statistics accumulate in f64.
#include "common.h"

#include <cstdlib>
#include <initializer_list>

namespace kdfm {
namespace {

constexpr int TT = 64;    // frames per tile
constexpr int CT = 64;    // channels per tile
constexpr int KMAX = 63;  // max kernel size

__global__ __launch_bounds__(256) void glu_mask_fwd_kernel(const float* __restrict__ a, const int64_t* __restrict__ lens,
                                                           float* __restrict__ g, int64_t rows, int64_t T, int64_t d) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * d) return;
  const int64_t r = idx / d, c = idx - r * d;
  const int64_t t = r % T, b = r / T;
  float v = 0.f;
  if (!lens || t < lens[b]) {
    const float x = a[r * 2 * d + c], y = a[r * 2 * d + d + c];
    v = x * sigmoidf_(y);
  }
  g[idx] = v;
}

// 16-byte-lane forms of the GLU mask kernels and the BN-SiLU forward (d % 4 == 0, aligned, fewer than 2^31
// float4 groups): 4 channels per thread and 32-bit index math -- the scalar kernels spend three 64-bit divisions per
// element (FastConformer-XL: 6 432 x 1024 GLU forward 35 us).  Same per-element arithmetic.
__device__ __forceinline__ float4 glu4(float4 x, float4 y) {
  return make_float4(x.x * sigmoidf_(y.x), x.y * sigmoidf_(y.y), x.z * sigmoidf_(y.z), x.w * sigmoidf_(y.w));
}

__global__ __launch_bounds__(256) void glu_mask_fwd4_kernel(const float* __restrict__ a, const int64_t* __restrict__ lens,
                                                            float* __restrict__ g, int n4, int T, int d4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int r = i / d4, c = i - r * d4;
  const int b = r / T, t = r - b * T;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!lens || t < lens[b]) {
    const float4* ar = reinterpret_cast<const float4*>(a) + (int64_t)r * 2 * d4;
    v = glu4(ar[c], ar[d4 + c]);
  }
  reinterpret_cast<float4*>(g)[i] = v;
}

template <typename O>
__global__ __launch_bounds__(256) void glu_mask_bwd4_kernel(const float* __restrict__ dg, const float* __restrict__ a,
                                                            const int64_t* __restrict__ lens, O* __restrict__ da, int n4,
                                                            int T, int d4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int r = i / d4, c = i - r * d4;
  const int b = r / T, t = r - b * T;
  float dx[4] = {0.f, 0.f, 0.f, 0.f}, dyv[4] = {0.f, 0.f, 0.f, 0.f};
  if (!lens || t < lens[b]) {
    const float4* ar = reinterpret_cast<const float4*>(a) + (int64_t)r * 2 * d4;
    const float4 x4 = ar[c], y4 = ar[d4 + c], g4 = reinterpret_cast<const float4*>(dg)[i];
    const float xs[4] = {x4.x, x4.y, x4.z, x4.w}, ys[4] = {y4.x, y4.y, y4.z, y4.w}, gs[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float s = sigmoidf_(ys[e]);
      dx[e] = gs[e] * s;
      dyv[e] = gs[e] * xs[e] * s * (1.f - s);
    }
  }
  const int64_t o = (int64_t)r * 2 * d4 * 4 + 4 * c;
  if constexpr (sizeof(O) == 2) {
    *reinterpret_cast<uint2*>(da + o) = make_uint2(pack_bf16x2(dx[0], dx[1]), pack_bf16x2(dx[2], dx[3]));
    *reinterpret_cast<uint2*>(da + o + 4 * d4) = make_uint2(pack_bf16x2(dyv[0], dyv[1]), pack_bf16x2(dyv[2], dyv[3]));
  } else {
    *reinterpret_cast<float4*>(da + o) = make_float4(dx[0], dx[1], dx[2], dx[3]);
    *reinterpret_cast<float4*>(da + o + 4 * d4) = make_float4(dyv[0], dyv[1], dyv[2], dyv[3]);
  }
}

template <typename O>
__global__ __launch_bounds__(256) void bn_silu_fwd4_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, const float* __restrict__ gm,
                                                           const float* __restrict__ bt, O* __restrict__ z, int n4,
                                                           int d4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int c = i % d4;
  const float4 yv = reinterpret_cast<const float4*>(y)[i], mu = reinterpret_cast<const float4*>(mean)[c];
  const float4 rs = reinterpret_cast<const float4*>(rstd)[c], g = reinterpret_cast<const float4*>(gm)[c];
  const float4 b = reinterpret_cast<const float4*>(bt)[c];
  const float o0 = siluf_(g.x * (yv.x - mu.x) * rs.x + b.x), o1 = siluf_(g.y * (yv.y - mu.y) * rs.y + b.y);
  const float o2 = siluf_(g.z * (yv.z - mu.z) * rs.z + b.z), o3 = siluf_(g.w * (yv.w - mu.w) * rs.w + b.w);
  if constexpr (sizeof(O) == 2)
    reinterpret_cast<uint2*>(z)[i] = make_uint2(pack_bf16x2(o0, o1), pack_bf16x2(o2, o3));
  else
    reinterpret_cast<float4*>(z)[i] = make_float4(o0, o1, o2, o3);
}

__host__ inline bool ew4_ok(int64_t rows, int64_t d, std::initializer_list<const void*> ptrs) {
  if (d % 4 || rows * (d / 4) >= ((int64_t)1 << 31)) return false;
  for (const void* p : ptrs)
    if (((uintptr_t)p) & 15) return false;
  return true;
}

template <typename O>   // uint16_t: da rounded to bf16 (kdfm_glu_mask_bwd_bf16)
__global__ __launch_bounds__(256) void glu_mask_bwd_kernel(const float* __restrict__ dg, const float* __restrict__ a,
                                                           const int64_t* __restrict__ lens, O* __restrict__ da,
                                                           int64_t rows, int64_t T, int64_t d) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * d) return;
  const int64_t r = idx / d, c = idx - r * d;
  const int64_t t = r % T, b = r / T;
  float dx = 0.f, dyv = 0.f;
  if (!lens || t < lens[b]) {
    const float x = a[r * 2 * d + c], y = a[r * 2 * d + d + c];
    const float s = sigmoidf_(y);
    const float gg = dg[idx];
    dx = gg * s;
    dyv = gg * x * s * (1.f - s);
  }
  if constexpr (sizeof(O) == 2) {
    da[r * 2 * d + c] = f2bf(dx);
    da[r * 2 * d + d + c] = f2bf(dyv);
  } else {
    da[r * 2 * d + c] = dx;
    da[r * 2 * d + d + c] = dyv;
  }
}

// Frame x channel tile staging shared by the depthwise-conv kernels: rows [t0 - pad, t0 + rows - pad)
// of one utterance, CT channels from c0, as float4 chunks (d % 4 == 0).  Every load of the tile is
// issued before the first LDS store, so the tile costs one memory round trip, not one per chunk: the
// loads are unconditional (frame and channel clamped into range) and masked by a multiply, since a
// conditional load is branched around and waited for one at a time.
constexpr int TQ = 8;  // float4 chunks per thread (rows <= TT + KMAX - 1 = 126)

__device__ __forceinline__ void tile_load(float4 (&v)[TQ], const float* __restrict__ src, int64_t b, int64_t t0,
                                          int pad, int rows, int64_t T, int64_t d, int64_t c0) {
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const int q = threadIdx.x + i * 256;
    const int rr = q >> 4, c4 = (q & 15) * 4;
    const int64_t t = t0 + rr - pad, c = c0 + c4;
    const bool ok = rr < rows && t >= 0 && t < T && c < d;
    const float m = ok ? 1.f : 0.f;
    const float4 x = *reinterpret_cast<const float4*>(src + (b * T + (ok ? t : 0)) * d + (ok ? c : 0));
    v[i] = make_float4(x.x * m, x.y * m, x.z * m, x.w * m);
  }
}

// the KC taps of channel c (zero past d), every load issued at once (channel clamped, masked by a
// multiply) before the tile's barrier: per-tap conditional loads inside the FMA loop were each
// waited for on their own
template <int KC>
__device__ __forceinline__ void taps_load(float (&wv)[KC], const float* __restrict__ w, int64_t c, int64_t d) {
  const bool ok = c < d;
  const float m = ok ? 1.f : 0.f;
  const float* wc = w + (ok ? c : 0) * KC;
#pragma unroll
  for (int k = 0; k < KC; ++k) wv[k] = wc[k] * m;
}

__device__ __forceinline__ void tile_store(const float4 (&v)[TQ], float* tile, int rows) {
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const int q = threadIdx.x + i * 256;
    const int rr = q >> 4, c4 = (q & 15) * 4;
    if (rr < rows) *reinterpret_cast<float4*>(tile + rr * CT + c4) = v[i];
  }
}

// y[b,t,c] = bias[c] + sum_k w[c,k] * g[b,t+k-pad,c]; stats[c] += (sum y, sum y^2)
// Lane = channel, wave = 16-frame group; with KC > 0 a 16-frame register window slides over the
// tile (one LDS read per 16 FMAs) with the taps in registers.
template <int KC>
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ y,
                                                         double* __restrict__ stats, int64_t T, int64_t d, int Krt) {
  constexpr int KM = KC > 0 ? KC : KMAX;
  __shared__ __attribute__((aligned(16))) float tile[(TT + KM - 1) * CT];
  __shared__ double red[2][4][CT];
  const int K = KC > 0 ? KC : Krt;
  const int pad = (K - 1) / 2;
  const int64_t b = blockIdx.z;
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int64_t c0 = (int64_t)blockIdx.y * CT;
  const int cc = threadIdx.x & 63;
  const int f0 = (threadIdx.x >> 6) * 16;
  const int64_t c = c0 + cc;
  const bool cok = c < d;
  float wv[KC > 0 ? KC : 1];
  float bc = 0.f;
  {
    float4 v[TQ];
    tile_load(v, g, b, t0, pad, TT + K - 1, T, d, c0);
    if constexpr (KC > 0) taps_load<KC>(wv, w, c, d);
    if (bias) bc = bias[cok ? c : 0] * (cok ? 1.f : 0.f);
    tile_store(v, tile, TT + K - 1);
  }
  __syncthreads();
  float acc[16];
#pragma unroll
  for (int tt = 0; tt < 16; ++tt) acc[tt] = bc;
  if constexpr (KC > 0) {
    float win[16];
#pragma unroll
    for (int tt = 0; tt < 16; ++tt) win[tt] = tile[(f0 + tt) * CT + cc];
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const float wk = wv[k];
#pragma unroll
      for (int tt = 0; tt < 16; ++tt) acc[tt] += wk * win[tt];
      if (k + 1 < KC) {
#pragma unroll
        for (int tt = 0; tt < 15; ++tt) win[tt] = win[tt + 1];
        win[15] = tile[(f0 + k + 16) * CT + cc];
      }
    }
  } else {
    for (int k = 0; k < K; ++k) {
      const float wk = cok ? w[c * K + k] : 0.f;
#pragma unroll
      for (int tt = 0; tt < 16; ++tt) acc[tt] += wk * tile[(f0 + tt + k) * CT + cc];
    }
  }
  double s1 = 0.0, s2 = 0.0;
  if (cok) {
#pragma unroll
    for (int tt = 0; tt < 16; ++tt) {
      const int64_t t = t0 + f0 + tt;
      if (t < T) {
        y[(b * T + t) * d + c] = acc[tt];
        s1 += acc[tt];
        s2 += (double)acc[tt] * acc[tt];
      }
    }
  }
  red[0][threadIdx.x >> 6][cc] = s1;
  red[1][threadIdx.x >> 6][cc] = s2;
  __syncthreads();
  if (stats && threadIdx.x < CT && c0 + threadIdx.x < d) {
    const int q = threadIdx.x;
    atomicAdd(stats + c0 + q, red[0][0][q] + red[0][1][q] + red[0][2][q] + red[0][3][q]);
    atomicAdd(stats + d + c0 + q, red[1][0][q] + red[1][1][q] + red[1][2][q] + red[1][3][q]);
  }
}

// Deterministic-mode BatchNorm statistics: stats[c] += sum_r y[r,c], stats[d+c] += sum_r y[r,c]^2 with
// one workgroup per 64 channels (lane = channel, the 4 waves stride the rows, fixed-order combine),
// replacing the per-tile f64 atomics of dwconv_fwd_kernel.
__global__ __launch_bounds__(256) void bn_stats_det_kernel(const float* __restrict__ y, double* __restrict__ stats,
                                                           int64_t rows, int64_t d) {
  __shared__ double sh[2][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  double s1 = 0.0, s2 = 0.0;
  if (c < d)
    for (int64_t r = w; r < rows; r += 4) {
      const double v = y[r * d + c];
      s1 += v;
      s2 += v * v;
    }
  sh[0][w][lane] = s1;
  sh[1][w][lane] = s2;
  __syncthreads();
  if (w == 0 && c < d) {
    stats[c] += (sh[0][0][lane] + sh[0][1][lane]) + (sh[0][2][lane] + sh[0][3][lane]);
    stats[d + c] += (sh[1][0][lane] + sh[1][1][lane]) + (sh[1][2][lane] + sh[1][3][lane]);
  }
}

// mean/rstd per channel: batch statistics (biased var) or running statistics (eval)
__global__ __launch_bounds__(256) void bn_finalize_kernel(const double* __restrict__ stats, const float* __restrict__ rm,
                                                          const float* __restrict__ rv, float* __restrict__ mean,
                                                          float* __restrict__ rstd, int64_t d, double count, float eps) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  if (stats) {
    const double m = stats[c] / count;
    double var = stats[d + c] / count - m * m;
    if (var < 0.0) var = 0.0;
    mean[c] = (float)m;
    rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  } else {
    mean[c] = rm[c];
    rstd[c] = rsqrtf(rv[c] + eps);
  }
}

// training step: batch mean/rstd AND the running-statistics update in one launch
__global__ __launch_bounds__(256) void bn_finalize_running_kernel(double* __restrict__ stats,
                                                                  float* __restrict__ rm, float* __restrict__ rv,
                                                                  float* __restrict__ mean, float* __restrict__ rstd,
                                                                  int64_t d, double count, float eps, float momentum) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  const double s1 = stats[c], s2 = stats[d + c];
  stats[c] = 0.0;   // reset for the next kdfm_dwconv_fwd accumulation (no memset launch per layer)
  stats[d + c] = 0.0;
  const double m = s1 / count;
  double var = s2 / count - m * m;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)m;
  rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
  rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * m);
  rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * unb);
}

__global__ __launch_bounds__(256) void bn_running_kernel(float* __restrict__ rm, float* __restrict__ rv,
                                                         const double* __restrict__ stats, int64_t d, double count,
                                                         float momentum) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  const double m = stats[c] / count;
  double var = stats[d + c] / count - m * m;
  if (var < 0.0) var = 0.0;
  const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
  rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * m);
  rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * unb);
}

// z = silu(gamma * (y - mean) * rstd + beta)
template <typename O>   // uint16_t: z rounded to bf16 (kdfm_bn_silu_fwd_bf16)
__global__ __launch_bounds__(256) void bn_silu_fwd_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, const float* __restrict__ gm,
                                                          const float* __restrict__ bt, O* __restrict__ z,
                                                          int64_t n, int64_t d) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n) return;
  const int64_t c = idx % d;
  const float pre = gm[c] * (y[idx] - mean[c]) * rstd[c] + bt[c];
  if constexpr (sizeof(O) == 2)
    z[idx] = f2bf(siluf_(pre));
  else
    z[idx] = siluf_(pre);
}

// red[c] += sum dyb ; red[d+c] += sum dyb * xhat, with dyb = dz * silu'(pre)
__global__ __launch_bounds__(256) void bn_silu_bwd_reduce_kernel(const float* __restrict__ dz, const float* __restrict__ y,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd,
                                                                 const float* __restrict__ gm, const float* __restrict__ bt,
                                                                 double* __restrict__ red, int64_t rows, int64_t d,
                                                                 int64_t rows_per) {
  __shared__ double sh[2][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = (r0 + rows_per < rows) ? r0 + rows_per : rows;
  double s1 = 0.0, s2 = 0.0;
  if (c < d) {
    const float mu = mean[c], rs = rstd[c], g = gm[c], b = bt[c];
    // 4 rows per wave per pass, their 8 loads issued together (clamped, masked): one dependent load per row made
    // the loop one memory round trip per row (13 us for 12 832 x 88); same per-row terms, same summation order
    int64_t r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      float yv[4], zv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        yv[u] = y[(r + 4 * u) * d + c];
        zv[u] = dz[(r + 4 * u) * d + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float xh = (yv[u] - mu) * rs;
        const float dyb = zv[u] * dsiluf_(g * xh + b);
        s1 += dyb;
        s2 += (double)dyb * xh;
      }
    }
    for (; r < r1; r += 4) {
      const float xh = (y[r * d + c] - mu) * rs;
      const float dyb = dz[r * d + c] * dsiluf_(g * xh + b);
      s1 += dyb;
      s2 += (double)dyb * xh;
    }
  }
  sh[0][w][lane] = s1;
  sh[1][w][lane] = s2;
  __syncthreads();
  if (w == 0 && c < d) {
    atomicAdd(red + c, sh[0][0][lane] + sh[0][1][lane] + sh[0][2][lane] + sh[0][3][lane]);
    atomicAdd(red + d + c, sh[1][0][lane] + sh[1][1][lane] + sh[1][2][lane] + sh[1][3][lane]);
  }
}

// dy = gamma*rstd*(dyb - mean(dyb) - xhat*mean(dyb*xhat))  (batch stats)   or gamma*rstd*dyb (eval)
__global__ __launch_bounds__(256) void bn_silu_bwd_apply_kernel(const float* __restrict__ dz, const float* __restrict__ y,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ gm,
                                                                const float* __restrict__ bt,
                                                                const double* __restrict__ red, float* __restrict__ dy,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                int64_t n, int64_t d, double count, int batch_stats,
                                                                double* __restrict__ red_next) {
  if (blockIdx.x == 0)   // the affine parameters' gradients (the reduction's totals): one launch fewer
    for (int64_t c = threadIdx.x; c < d; c += 256) {
      dgamma[c] += (float)red[d + c];
      dbeta[c] += (float)red[c];
      if (red_next) {   // the next call's sums start at zero without a memset launch (kdfm_bn_silu_bwd2)
        red_next[c] = 0.0;
        red_next[d + c] = 0.0;
      }
    }
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n) return;
  const int64_t c = idx % d;
  const float xh = (y[idx] - mean[c]) * rstd[c];
  const float dyb = dz[idx] * dsiluf_(gm[c] * xh + bt[c]);
  float v;
  if (batch_stats) {
    const float m1 = (float)(red[c] / count), m2 = (float)(red[d + c] / count);
    v = gm[c] * rstd[c] * (dyb - m1 - xh * m2);
  } else {
    v = gm[c] * rstd[c] * dyb;
  }
  dy[idx] = v;
}

// BatchNorm + SiLU backward applied on load (kdfm_dwconv_bwd_bn): the depthwise backward's input gradient
//   dy = gamma rstd (dz silu'(gamma xh + beta) - m1 - xh m2),  xh = (y - mean) rstd,  m1|m2 = red / count
// (batch statistics; gamma rstd dz silu'(.) with the running ones) is formed from dz and y as the tile is
// staged, so it never reaches HBM and its elementwise launch disappears.
struct BnApply {
  const float* y; const float* mean; const float* rstd; const float* gm; const float* bt; const double* red;
  double count; int batch_stats;
  float* dgamma; float* dbeta; double* red_next;   // block (0,0,0): affine grads from red, zero red_next
};

__device__ __forceinline__ void tile_load_bn(float4 (&v)[TQ], const float* __restrict__ dz, const BnApply& a,
                                             int64_t b, int64_t t0, int pad, int rows, int64_t T, int64_t d,
                                             int64_t c0) {
  // this thread's 4 channels are the same for every unit (256 threads, 16 float4 per tile row)
  const int c4 = (threadIdx.x & 15) * 4;
  const int64_t cb = c0 + c4 < d ? c0 + c4 : 0;
  float mu[4], rs[4], gm[4], bt[4], m1[4], m2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mu[j] = a.mean[cb + j];
    rs[j] = a.rstd[cb + j];
    gm[j] = a.gm[cb + j];
    bt[j] = a.bt[cb + j];
    m1[j] = a.batch_stats ? (float)(a.red[cb + j] / a.count) : 0.f;
    m2[j] = a.batch_stats ? (float)(a.red[d + cb + j] / a.count) : 0.f;
  }
  float4 z[TQ], yv[TQ];
  float mk[TQ];
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const int q = threadIdx.x + i * 256;
    const int rr = q >> 4;
    const int64_t t = t0 + rr - pad, c = c0 + c4;
    const bool ok = rr < rows && t >= 0 && t < T && c < d;
    mk[i] = ok ? 1.f : 0.f;
    const int64_t off = (b * T + (ok ? t : 0)) * d + (ok ? c : 0);
    z[i] = *reinterpret_cast<const float4*>(dz + off);
    yv[i] = *reinterpret_cast<const float4*>(a.y + off);
  }
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const float zz[4] = {z[i].x, z[i].y, z[i].z, z[i].w};
    const float yy[4] = {yv[i].x, yv[i].y, yv[i].z, yv[i].w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (yy[j] - mu[j]) * rs[j];
      const float dyb = zz[j] * dsiluf_(gm[j] * xh + bt[j]);
      o[j] = gm[j] * rs[j] * (dyb - m1[j] - xh * m2[j]) * mk[i];
    }
    v[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// Backward of the depthwise conv over one (TT frames x CT channels) tile of one utterance:
//   dg[b,t,c] = sum_k w[c,k] * dy[b,t-k+pad,c]
//   dw[c,k]  += sum_t dy[b,t,c] * g[b,t+k-pad,c],   db[c] += sum_t dy[b,t,c]
// Lane = channel, wave = a 16-frame group.  With the kernel size known at compile time (KC > 0)
// both sums run from register sliding windows (one LDS read per 16..K FMAs); KC == 0 is the
// runtime-K path.  Weight/bias sums land in part[(b*ntt + tile)][c*K + k | d*K + c] and are folded
// by launch_colsum on the host side (no hot atomics).
template <int KC, bool BN = false>
__global__ __launch_bounds__(256) void dwconv_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ g,
                                                         const float* __restrict__ w, float* __restrict__ dg,
                                                         float* __restrict__ part, int64_t T, int64_t d, int Krt,
                                                         BnApply bn) {
  constexpr int KM = KC > 0 ? KC : KMAX;
  __shared__ __attribute__((aligned(16))) float tdy[(TT + KM - 1) * CT];  // frames t0-pad .. t0+TT-1+pad
  __shared__ __attribute__((aligned(16))) float tg[(TT + KM - 1) * CT];
  // KC > 0: one partial slot per wave, folded in wave order below (deterministic); the runtime-K
  // path keeps LDS atomics (not used by the k = 15 / 31 configurations)
  constexpr int NSLOT = KC > 0 ? 4 : 1;
  __shared__ float red[NSLOT][(KM + 1) * CT];
  const int K = KC > 0 ? KC : Krt;
  const int pad = (K - 1) / 2;
  const int64_t b = blockIdx.z;
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int64_t c0 = (int64_t)blockIdx.y * CT;
  const int rowsIn = TT + K - 1;
  const int slot = KC > 0 ? (threadIdx.x >> 6) : 0;
  const int cc = threadIdx.x & 63;
  const int f0 = (threadIdx.x >> 6) * 16;  // this wave's first frame in the tile
  const int64_t c = c0 + cc;
  const bool cok = c < d;
  float wv[KC > 0 ? KC : 1];
  {
    float4 v1[TQ], v2[TQ];
    if constexpr (BN) {
      tile_load_bn(v1, dy, bn, b, t0, pad, rowsIn, T, d, c0);   // dy here is dz: the BN-SiLU input gradient
    } else {
      tile_load(v1, dy, b, t0, pad, rowsIn, T, d, c0);
    }
    tile_load(v2, g, b, t0, pad, rowsIn, T, d, c0);
    if (BN && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      for (int64_t ch = threadIdx.x; ch < d; ch += 256) {   // the BatchNorm affine gradients (the reduction's totals)
        bn.dgamma[ch] += (float)bn.red[d + ch];
        bn.dbeta[ch] += (float)bn.red[ch];
        if (bn.red_next) {
          bn.red_next[ch] = 0.0;
          bn.red_next[d + ch] = 0.0;
        }
      }
    }
    if constexpr (KC > 0) taps_load<KC>(wv, w, c, d);
    tile_store(v1, tdy, rowsIn);
    tile_store(v2, tg, rowsIn);
  }
  for (int e = threadIdx.x; e < NSLOT * (K + 1) * CT; e += 256) (&red[0][0])[e] = 0.f;
  __syncthreads();
  float bsum = 0.f;
  if constexpr (KC > 0) {
    // Sliding 16-frame register windows with the tap loop outermost: every register index is a
    // compile-time constant (a data-dependent tap index would make the compiler fall back to
    // VGPR-indexed moves).  Tile row r <-> frame t0 + r - pad.
    // dg[f0+tt] = sum_k w[K-1-kk] * tdy[f0 + tt + kk]   (kk = K-1-k)
    float win[16], acc[16];
#pragma unroll
    for (int tt = 0; tt < 16; ++tt) {
      win[tt] = tdy[(f0 + tt) * CT + cc];
      acc[tt] = 0.f;
    }
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const float wk = wv[KC - 1 - kk];
#pragma unroll
      for (int tt = 0; tt < 16; ++tt) acc[tt] += wk * win[tt];
      if (kk + 1 < KC) {
#pragma unroll
        for (int tt = 0; tt < 15; ++tt) win[tt] = win[tt + 1];
        win[15] = tdy[(f0 + kk + 16) * CT + cc];
      }
    }
    if (cok) {
#pragma unroll
      for (int tt = 0; tt < 16; ++tt) {
        const int64_t t = t0 + f0 + tt;
        if (t < T) dg[(b * T + t) * d + c] = acc[tt];
      }
    }
    // dw[k] = sum_tt dy[f0+tt] * tg[f0 + tt + k]
    float dyr[16];
#pragma unroll
    for (int tt = 0; tt < 16; ++tt) {
      dyr[tt] = tdy[(f0 + tt + pad) * CT + cc];
      bsum += dyr[tt];
      win[tt] = tg[(f0 + tt) * CT + cc];
    }
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      float s = 0.f;
#pragma unroll
      for (int tt = 0; tt < 16; ++tt) s += dyr[tt] * win[tt];
      red[slot][k * CT + cc] = s;
      if (k + 1 < KC) {
#pragma unroll
        for (int tt = 0; tt < 15; ++tt) win[tt] = win[tt + 1];
        win[15] = tg[(f0 + k + 16) * CT + cc];
      }
    }
  } else {
    for (int tt = 0; tt < 16; ++tt) {
      const int64_t t = t0 + f0 + tt;
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc += (cok ? w[c * K + k] : 0.f) * tdy[(f0 + tt + K - 1 - k) * CT + cc];
      if (cok && t < T) dg[(b * T + t) * d + c] = acc;
      bsum += tdy[(f0 + tt + pad) * CT + cc];
    }
    for (int k = 0; k < K; ++k) {
      float acc = 0.f;
      for (int tt = 0; tt < 16; ++tt) acc += tdy[(f0 + tt + pad) * CT + cc] * tg[(f0 + tt + k) * CT + cc];
      atomicAdd(&red[0][k * CT + cc], acc);
    }
  }
  if constexpr (KC > 0)
    red[slot][K * CT + cc] = bsum;
  else
    atomicAdd(&red[0][K * CT + cc], bsum);
  __syncthreads();
  const int64_t ld = d * (K + 1);
  float* pr = part + (b * gridDim.x + blockIdx.x) * ld;
  for (int e = threadIdx.x; e < (K + 1) * CT; e += 256) {
    const int q = e / (K + 1), k = e % (K + 1);
    const int64_t cq = c0 + q;
    if (cq >= d) continue;
    float v = red[0][k * CT + q];
    if constexpr (KC > 0) v = (v + red[1][k * CT + q]) + (red[2][k * CT + q] + red[3][k * CT + q]);
    if (k < K)
      pr[cq * K + k] = v;
    else
      pr[d * K + cq] = v;
  }
}

// The same backward with a lane owning a channel PAIR (channels c0 + 2 lane, +1: 128 channels per workgroup,
// 8-byte LDS window reads, every FMA a packed v_pk_fma_f32 over the two channels).  The Conformer's d = 88 took
// 2 channel tiles of 64 (the second 24/64 used) and 1 792 waves at 160 VGPRs (1.75 per SIMD, contending for
// issue); here d <= 128 is one tile: 224 workgroups x 4 waves at the bench shape, each wave's instruction
// count about that of one wave before.  Per output element the same operations in the same order as
// dwconv_bwd_kernel (the tap chain of dg, the frame chain of each dw tap, the wave-slot combine, the BN
// apply): bitwise its results.  The dw reduction reuses the tile LDS after the last window read.
constexpr int CP = 128;   // channels per workgroup (64 lanes x 2)
// Channel pairs for d <= 128 (one workgroup column): the d = 88 backward with BN-SiLU on load 20.3 -> 16.6 us
// isolated (profiles/r06/r6an); at d = 176 the 128 + 48 split is slower than the one-channel kernel's 64 + 64 + 48
// tiles (29.4 -> 36.6 us).  The forward only without the fused f64 statistics (7.7 -> 7.2 us; with them 10.8 ->
// 11.6 us: two channels' f64 sums per lane).  KDFM_DWC_P2=0: never, =2: always (read per call: tests compare)
inline int dwc_mode() {
  const char* e = getenv("KDFM_DWC_P2");
  return e ? atoi(e) : 1;
}
inline bool dwc_p2(int64_t d, bool fused_stats = false) {
  const int m = dwc_mode();
  return m == 2 || (m == 1 && d <= CP && !fused_stats);
}
typedef float pf2 __attribute__((ext_vector_type(2)));

template <int KC>
constexpr int p2_rows() { return TT + KC - 1; }
template <int KC, int NT>
constexpr int p2_tq() { return (p2_rows<KC>() * (CP / 4) + NT - 1) / NT; }

template <int KC, int NT>
__device__ __forceinline__ void p2_tile_load(float4 (&v)[(p2_tq<KC, NT>())], const float* __restrict__ src, int64_t b,
                                             int64_t t0, int64_t T, int64_t d, int64_t c0) {
  constexpr int pad = (KC - 1) / 2, rows = p2_rows<KC>();
#pragma unroll
  for (int i = 0; i < p2_tq<KC, NT>(); ++i) {
    const int q = threadIdx.x + i * NT;
    const int rr = q >> 5, c4 = (q & 31) * 4;
    const int64_t t = t0 + rr - pad, c = c0 + c4;
    const bool ok = rr < rows && t >= 0 && t < T && c < d;
    const float m = ok ? 1.f : 0.f;
    const float4 x = *reinterpret_cast<const float4*>(src + (b * T + (ok ? t : 0)) * d + (ok ? c : 0));
    v[i] = make_float4(x.x * m, x.y * m, x.z * m, x.w * m);
  }
}

template <int KC, int NT>
__device__ __forceinline__ void p2_tile_store(const float4 (&v)[(p2_tq<KC, NT>())], float* tile) {
  constexpr int rows = p2_rows<KC>();
#pragma unroll
  for (int i = 0; i < p2_tq<KC, NT>(); ++i) {
    const int q = threadIdx.x + i * NT;
    const int rr = q >> 5, c4 = (q & 31) * 4;
    if (rr < rows) *reinterpret_cast<float4*>(tile + rr * CP + c4) = v[i];
  }
}

// Forward with a lane owning a channel pair (as dwconv_bwd_p2_kernel), 8 waves of 8 frames: y = bias + the tap
// chain in dwconv_fwd_kernel's order (bitwise its y); the BatchNorm sums per channel in f64, this wave's frames in
// order, the 8 waves added in order before the one atomic per channel and workgroup.
constexpr int P2_NT = 512;
template <int KC>
__global__ __launch_bounds__(P2_NT) void dwconv_fwd_p2_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ y,
                                                              double* __restrict__ stats, int64_t T, int64_t d) {
  constexpr int rows = p2_rows<KC>(), TQW = p2_tq<KC, P2_NT>(), FW = TT / 8;
  __shared__ __attribute__((aligned(16))) float tile[rows * CP];
  __shared__ double red[2][8][CP];
  const int64_t b = blockIdx.z;
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int64_t c0 = (int64_t)blockIdx.y * CP;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f0 = wave * FW;
  const int64_t c = c0 + 2 * lane;
  const bool cok = c < d;
  pf2 wv[KC];
  pf2 bc = pf2{0.f, 0.f};
  {
    float4 v[TQW];
    p2_tile_load<KC, P2_NT>(v, g, b, t0, T, d, c0);
    const float mm = cok ? 1.f : 0.f;
    const float* wa = w + (cok ? c : 0) * KC;
    const float* wb = w + (cok ? c + 1 : 0) * KC;
#pragma unroll
    for (int k = 0; k < KC; ++k) wv[k] = pf2{wa[k] * mm, wb[k] * mm};
    if (bias) bc = pf2{bias[cok ? c : 0] * mm, bias[cok ? c + 1 : 0] * mm};
    p2_tile_store<KC, P2_NT>(v, tile);
  }
  __syncthreads();
  auto rd = [&](int r) { return *reinterpret_cast<const pf2*>(tile + r * CP + 2 * lane); };
  pf2 acc[FW], win[FW];
#pragma unroll
  for (int tt = 0; tt < FW; ++tt) {
    acc[tt] = bc;
    win[tt] = rd(f0 + tt);
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const pf2 wk = wv[k];
#pragma unroll
    for (int tt = 0; tt < FW; ++tt) acc[tt] = __builtin_elementwise_fma(wk, win[tt], acc[tt]);
    if (k + 1 < KC) {
#pragma unroll
      for (int tt = 0; tt < FW - 1; ++tt) win[tt] = win[tt + 1];
      win[FW - 1] = rd(f0 + k + FW);
    }
  }
  double s1a = 0.0, s2a = 0.0, s1b = 0.0, s2b = 0.0;
  if (cok) {
#pragma unroll
    for (int tt = 0; tt < FW; ++tt) {
      const int64_t t = t0 + f0 + tt;
      if (t < T) {
        *reinterpret_cast<pf2*>(y + (b * T + t) * d + c) = acc[tt];
        s1a += acc[tt].x;
        s2a += (double)acc[tt].x * acc[tt].x;
        s1b += acc[tt].y;
        s2b += (double)acc[tt].y * acc[tt].y;
      }
    }
  }
  if (!stats) return;
  red[0][wave][2 * lane] = s1a;
  red[0][wave][2 * lane + 1] = s1b;
  red[1][wave][2 * lane] = s2a;
  red[1][wave][2 * lane + 1] = s2b;
  __syncthreads();
  if (threadIdx.x < 2 * CP && c0 + (threadIdx.x & (CP - 1)) < d) {
    const int q = threadIdx.x & (CP - 1), m = threadIdx.x >> 7;   // m: sum (0) or sum of squares (1)
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += red[m][i][q];
    atomicAdd(stats + m * d + c0 + q, v);
  }
}

// 8 waves: waves 0-3 form dg of frame groups 0-3, waves 4-7 the dw / db sums of the same groups -- each wave half the
// serial chain of a 4-wave workgroup's, two waves per SIMD, and no sum regrouped (bitwise as before)
template <int KC, bool BN>
__global__ __launch_bounds__(P2_NT) void dwconv_bwd_p2_kernel(const float* __restrict__ dy, const float* __restrict__ g,
                                                              const float* __restrict__ w, float* __restrict__ dg,
                                                              float* __restrict__ part, int64_t T, int64_t d, BnApply bn) {
  constexpr int K = KC, pad = (KC - 1) / 2, rows = p2_rows<KC>(), TQW = p2_tq<KC, P2_NT>();
  __shared__ __attribute__((aligned(16))) float lds[2 * rows * CP];
  float* tdy = lds;
  float* tg = lds + rows * CP;
  const int64_t b = blockIdx.z;
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int64_t c0 = (int64_t)blockIdx.y * CP;
  const int lane = threadIdx.x & 63, slot = (threadIdx.x >> 6) & 3;
  const bool dwave = threadIdx.x >= 256;   // a dw / db wave
  const int f0 = slot * 16;   // this wave's first frame in the tile
  const int64_t c = c0 + 2 * lane;
  const bool cok = c < d;     // d % 4 == 0: a pair is wholly in or out
  pf2 wv[KC];
  {
    float4 v1[TQW], v2[TQW];
    if constexpr (BN) {
      // BN + SiLU backward applied on load (tile_load_bn over 128-channel rows)
      const int c4 = (threadIdx.x & 31) * 4;
      const int64_t cb = c0 + c4 < d ? c0 + c4 : 0;
      float mu[4], rs[4], gm[4], bt[4], m1[4], m2[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mu[j] = bn.mean[cb + j];
        rs[j] = bn.rstd[cb + j];
        gm[j] = bn.gm[cb + j];
        bt[j] = bn.bt[cb + j];
        m1[j] = bn.batch_stats ? (float)(bn.red[cb + j] / bn.count) : 0.f;
        m2[j] = bn.batch_stats ? (float)(bn.red[d + cb + j] / bn.count) : 0.f;
      }
      float4 z[TQW], yv[TQW];
      float mk[TQW];
#pragma unroll
      for (int i = 0; i < TQW; ++i) {
        const int q = threadIdx.x + i * P2_NT;
        const int rr = q >> 5;
        const int64_t t = t0 + rr - pad, cc = c0 + c4;
        const bool ok = rr < rows && t >= 0 && t < T && cc < d;
        mk[i] = ok ? 1.f : 0.f;
        const int64_t off = (b * T + (ok ? t : 0)) * d + (ok ? cc : 0);
        z[i] = *reinterpret_cast<const float4*>(dy + off);
        yv[i] = *reinterpret_cast<const float4*>(bn.y + off);
      }
      p2_tile_load<KC, P2_NT>(v2, g, b, t0, T, d, c0);
#pragma unroll
      for (int i = 0; i < TQW; ++i) {
        const float zz[4] = {z[i].x, z[i].y, z[i].z, z[i].w};
        const float yy[4] = {yv[i].x, yv[i].y, yv[i].z, yv[i].w};
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (yy[j] - mu[j]) * rs[j];
          const float dyb = zz[j] * dsiluf_(gm[j] * xh + bt[j]);
          o[j] = gm[j] * rs[j] * (dyb - m1[j] - xh * m2[j]) * mk[i];
        }
        v1[i] = make_float4(o[0], o[1], o[2], o[3]);
      }
      if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
        for (int64_t ch = threadIdx.x; ch < d; ch += P2_NT) {
          bn.dgamma[ch] += (float)bn.red[d + ch];
          bn.dbeta[ch] += (float)bn.red[ch];
          if (bn.red_next) {
            bn.red_next[ch] = 0.0;
            bn.red_next[d + ch] = 0.0;
          }
        }
      }
    } else {
      p2_tile_load<KC, P2_NT>(v1, dy, b, t0, T, d, c0);
      p2_tile_load<KC, P2_NT>(v2, g, b, t0, T, d, c0);
    }
    {   // the taps of the lane's two channels (zero past d)
      const float mm = cok ? 1.f : 0.f;
      const float* wa = w + (cok ? c : 0) * KC;
      const float* wb = w + (cok ? c + 1 : 0) * KC;
#pragma unroll
      for (int k = 0; k < KC; ++k) wv[k] = pf2{wa[k] * mm, wb[k] * mm};
    }
    p2_tile_store<KC, P2_NT>(v1, tdy);
    p2_tile_store<KC, P2_NT>(v2, tg);
  }
  __syncthreads();
  auto rd = [&](const float* tile, int r) { return *reinterpret_cast<const pf2*>(tile + r * CP + 2 * lane); };
  pf2 sk[KC];
  pf2 bsum = pf2{0.f, 0.f};
  if (!dwave) {
  // dg[f0+tt] = sum_kk w[K-1-kk] * tdy[f0 + tt + kk]
  pf2 win[16], acc[16];
#pragma unroll
  for (int tt = 0; tt < 16; ++tt) {
    win[tt] = rd(tdy, f0 + tt);
    acc[tt] = pf2{0.f, 0.f};
  }
#pragma unroll
  for (int kk = 0; kk < KC; ++kk) {
    const pf2 wk = wv[KC - 1 - kk];
#pragma unroll
    for (int tt = 0; tt < 16; ++tt) acc[tt] = __builtin_elementwise_fma(wk, win[tt], acc[tt]);
    if (kk + 1 < KC) {
#pragma unroll
      for (int tt = 0; tt < 15; ++tt) win[tt] = win[tt + 1];
      win[15] = rd(tdy, f0 + kk + 16);
    }
  }
  if (cok) {
#pragma unroll
    for (int tt = 0; tt < 16; ++tt) {
      const int64_t t = t0 + f0 + tt;
      if (t < T) *reinterpret_cast<pf2*>(dg + (b * T + t) * d + c) = acc[tt];
    }
  }
  } else {
  // dw[k] = sum_tt dy[f0+tt] * tg[f0 + tt + k]; db = sum_tt dy[f0+tt].  Frames outermost, a KC-row window of tg
  // sliding down them: the KC tap sums are independent chains (a tap's 16-frame chain back to back would stall
  // the packed FMA's dependency latency), each still summed over tt in order
  pf2 wg[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    wg[k] = rd(tg, f0 + k);
    sk[k] = pf2{0.f, 0.f};
  }
#pragma unroll
  for (int tt = 0; tt < 16; ++tt) {
    const pf2 dyv = rd(tdy, f0 + tt + pad);
    bsum += dyv;
#pragma unroll
    for (int k = 0; k < KC; ++k) sk[k] = __builtin_elementwise_fma(dyv, wg[k], sk[k]);
    if (tt + 1 < 16) {
#pragma unroll
      for (int k = 0; k < KC - 1; ++k) wg[k] = wg[k + 1];
      wg[KC - 1] = rd(tg, f0 + tt + KC);
    }
  }
  }
  __syncthreads();   // every wave is past its last tile read: the tiles' LDS takes the wave slots
  float* red = lds;  // red[slot][k][CP], k = K: the bias sums
  if (dwave) {
#pragma unroll
    for (int k = 0; k < KC; ++k) *reinterpret_cast<pf2*>(red + (slot * (K + 1) + k) * CP + 2 * lane) = sk[k];
    *reinterpret_cast<pf2*>(red + (slot * (K + 1) + K) * CP + 2 * lane) = bsum;
  }
  __syncthreads();
  const int64_t ld = d * (K + 1);
  float* pr = part + (b * gridDim.x + blockIdx.x) * ld;
  for (int e = threadIdx.x; e < (K + 1) * CP; e += P2_NT) {
    const int q = e / (K + 1), k = e % (K + 1);
    const int64_t cq = c0 + q;
    if (cq >= d) continue;
    const float* rq = red + k * CP + q;
    const int sl = (K + 1) * CP;
    const float v = (rq[0] + rq[sl]) + (rq[2 * sl] + rq[3 * sl]);
    if (k < K)
      pr[cq * K + k] = v;
    else
      pr[d * K + cq] = v;
  }
}

}  // namespace
}  // namespace kdfm


extern "C" {

int kdfm_glu_mask_fwd(const float* a, const int64_t* lengths, float* g, int64_t B, int64_t T, int64_t d,
                      void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(a && g, "null pointer");
  const int64_t n = B * T * d;
  if (n == 0) return KDFM_OK;
  if (ew4_ok(B * T, d, {a, g}) && T < ((int64_t)1 << 31)) {
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(glu_mask_fwd4_kernel, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), a,
                       lengths, g, (int)n4, (int)T, (int)(d / 4));
    return check_launch("kdfm_glu_mask_fwd");
  }
  hipLaunchKernelGGL(glu_mask_fwd_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), a,
                     lengths, g, B * T, T, d);
  return check_launch("kdfm_glu_mask_fwd");
}

int kdfm_glu_mask_bwd(const float* dg, const float* a, const int64_t* lengths, float* da, int64_t B, int64_t T,
                      int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dg && a && da, "null pointer");
  const int64_t n = B * T * d;
  if (n == 0) return KDFM_OK;
  if (ew4_ok(B * T, d, {dg, a, da})) {
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(glu_mask_bwd4_kernel<float>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), dg,
                       a, lengths, da, (int)n4, (int)T, (int)(d / 4));
    return check_launch("kdfm_glu_mask_bwd");
  }
  hipLaunchKernelGGL(glu_mask_bwd_kernel<float>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), dg,
                     a, lengths, da, B * T, T, d);
  return check_launch("kdfm_glu_mask_bwd");
}

int kdfm_glu_mask_bwd_bf16(const float* dg, const float* a, const int64_t* lengths, uint16_t* da, int64_t B,
                           int64_t T, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dg && a && da, "null pointer");
  const int64_t n = B * T * d;
  if (n == 0) return KDFM_OK;
  if (ew4_ok(B * T, d, {dg, a, da})) {
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(glu_mask_bwd4_kernel<uint16_t>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), dg,
                       a, lengths, da, (int)n4, (int)T, (int)(d / 4));
    return check_launch("kdfm_glu_mask_bwd");
  }
  hipLaunchKernelGGL(glu_mask_bwd_kernel<uint16_t>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream),
                     dg, a, lengths, da, B * T, T, d);
  return check_launch("kdfm_glu_mask_bwd_bf16");
}


int kdfm_dwconv_fwd(const float* g, const float* w, const float* bias, float* y, double* stats, int64_t B, int64_t T,
                    int64_t d, int64_t K, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(g && w && y, "null pointer");
  KDFM_REQUIRE(K >= 1 && K <= KMAX && (K % 2) == 1, "kernel size must be odd and <= 63");
  KDFM_REQUIRE(d % 4 == 0 && (((uintptr_t)g) & 15) == 0, "channels must be a multiple of 4, input 16-B aligned");
  if (B * T * d == 0) return KDFM_OK;
  dim3 grid((unsigned)ceil_div(T, TT), (unsigned)ceil_div(d, CT), (unsigned)B);
  double* st_fused = deterministic() ? nullptr : stats;
  if (dwc_p2(d, st_fused != nullptr) && (K == 31 || K == 15 || K == 9)) {
    const dim3 g2((unsigned)ceil_div(T, TT), (unsigned)ceil_div(d, CP), (unsigned)B);
    if (K == 31)
      hipLaunchKernelGGL(dwconv_fwd_p2_kernel<31>, g2, dim3(P2_NT), 0, as_stream(stream), g, w, bias, y, st_fused, T, d);
    else if (K == 9)
      hipLaunchKernelGGL(dwconv_fwd_p2_kernel<9>, g2, dim3(P2_NT), 0, as_stream(stream), g, w, bias, y, st_fused, T, d);
    else
      hipLaunchKernelGGL(dwconv_fwd_p2_kernel<15>, g2, dim3(P2_NT), 0, as_stream(stream), g, w, bias, y, st_fused, T, d);
  } else if (K == 31)
    hipLaunchKernelGGL(dwconv_fwd_kernel<31>, grid, dim3(256), 0, as_stream(stream), g, w, bias, y, st_fused, T, d, (int)K);
  else if (K == 9)   // FastConformer(-XL), fast-conformer_ctc_bpe.yaml conv_kernel_size 9
    hipLaunchKernelGGL(dwconv_fwd_kernel<9>, grid, dim3(256), 0, as_stream(stream), g, w, bias, y, st_fused, T, d, (int)K);
  else if (K == 15)
    hipLaunchKernelGGL(dwconv_fwd_kernel<15>, grid, dim3(256), 0, as_stream(stream), g, w, bias, y, st_fused, T, d, (int)K);
  else
    hipLaunchKernelGGL(dwconv_fwd_kernel<0>, grid, dim3(256), 0, as_stream(stream), g, w, bias, y, st_fused, T, d, (int)K);
  int rc = check_launch("kdfm_dwconv_fwd");
  if (rc || !stats || st_fused) return rc;
  hipLaunchKernelGGL(bn_stats_det_kernel, dim3((unsigned)ceil_div(d, 64)), dim3(256), 0, as_stream(stream), y, stats,
                     B * T, d);
  return check_launch("kdfm_dwconv_fwd(det stats)");
}

int64_t kdfm_dwconv_bwd_ws(int64_t B, int64_t T, int64_t d, int64_t K) {
  return B * kdfm::ceil_div(T, kdfm::TT) * d * (K + 1);
}

int kdfm_dwconv_bwd(const float* dy, const float* g, const float* w, float* dg, float* dw, float* db, float* ws,
                    int64_t B, int64_t T, int64_t d, int64_t K, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && g && w && dg && ws, "null pointer");
  KDFM_REQUIRE((dw == nullptr) == (db == nullptr), "dw and db: both or neither");
  KDFM_REQUIRE(K >= 1 && K <= KMAX && (K % 2) == 1, "kernel size must be odd and <= 63");
  KDFM_REQUIRE(d % 4 == 0 && ((((uintptr_t)g) | ((uintptr_t)dy)) & 15) == 0,
               "channels must be a multiple of 4, inputs 16-B aligned");
  if (B * T * d == 0) return KDFM_OK;
  static_assert(TT == 64, "dwconv_bwd assumes 4 waves x 16 frames per tile");
  hipStream_t st = as_stream(stream);
  const int64_t ntt = ceil_div(T, TT);
  dim3 grid((unsigned)ntt, (unsigned)ceil_div(d, CT), (unsigned)B);
  const BnApply none{};
  if (dwc_p2(d) && (K == 31 || K == 15 || K == 9)) {
    const dim3 g2((unsigned)ntt, (unsigned)ceil_div(d, CP), (unsigned)B);
    if (K == 31)
      hipLaunchKernelGGL((dwconv_bwd_p2_kernel<31, false>), g2, dim3(P2_NT), 0, st, dy, g, w, dg, ws, T, d, none);
    else if (K == 15)
      hipLaunchKernelGGL((dwconv_bwd_p2_kernel<15, false>), g2, dim3(P2_NT), 0, st, dy, g, w, dg, ws, T, d, none);
    else
      hipLaunchKernelGGL((dwconv_bwd_p2_kernel<9, false>), g2, dim3(P2_NT), 0, st, dy, g, w, dg, ws, T, d, none);
  } else if (K == 31)
    hipLaunchKernelGGL(dwconv_bwd_kernel<31>, grid, dim3(256), 0, st, dy, g, w, dg, ws, T, d, (int)K, none);
  else if (K == 9)
    hipLaunchKernelGGL(dwconv_bwd_kernel<9>, grid, dim3(256), 0, st, dy, g, w, dg, ws, T, d, (int)K, none);
  else if (K == 15)
    hipLaunchKernelGGL(dwconv_bwd_kernel<15>, grid, dim3(256), 0, st, dy, g, w, dg, ws, T, d, (int)K, none);
  else
    hipLaunchKernelGGL(dwconv_bwd_kernel<0>, grid, dim3(256), 0, st, dy, g, w, dg, ws, T, d, (int)K, none);
  int rc = check_launch("kdfm_dwconv_bwd");
  if (rc || !dw) return rc;   // dw == db == NULL: the partials stay in ws for kdfm_dwconv_bwd_fold
  return kdfm_dwconv_bwd_fold(ws, dw, db, B, T, d, K, stream);
}

int kdfm_dwconv_bwd_bn(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, const double* red, double* red_next, float* dgamma, float* dbeta,
                       int32_t batch_stats, const float* g, const float* w, float* dg, float* ws, int64_t B,
                       int64_t T, int64_t d, int64_t K, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dz && y && mean && rstd && gamma && beta && red && dgamma && dbeta && g && w && dg && ws,
               "null pointer");
  KDFM_REQUIRE(K == 31 || K == 15 || K == 9, "BN-applied depthwise backward: kernel size 9, 15 or 31");
  KDFM_REQUIRE(d % 4 == 0 && ((((uintptr_t)g) | ((uintptr_t)dz) | ((uintptr_t)y)) & 15) == 0,
               "channels must be a multiple of 4, inputs 16-B aligned");
  KDFM_REQUIRE(red_next != red, "red_next must be another buffer");
  if (B * T * d == 0) return KDFM_OK;
  hipStream_t st = as_stream(stream);
  const int64_t ntt = ceil_div(T, TT);
  dim3 grid((unsigned)ntt, (unsigned)ceil_div(d, CT), (unsigned)B);
  const BnApply bn{y, mean, rstd, gamma, beta, red, (double)(B * T), batch_stats, dgamma, dbeta, red_next};
  if (dwc_p2(d)) {
    const dim3 g2((unsigned)ntt, (unsigned)ceil_div(d, CP), (unsigned)B);
    if (K == 31)
      hipLaunchKernelGGL((dwconv_bwd_p2_kernel<31, true>), g2, dim3(P2_NT), 0, st, dz, g, w, dg, ws, T, d, bn);
    else if (K == 9)
      hipLaunchKernelGGL((dwconv_bwd_p2_kernel<9, true>), g2, dim3(P2_NT), 0, st, dz, g, w, dg, ws, T, d, bn);
    else
      hipLaunchKernelGGL((dwconv_bwd_p2_kernel<15, true>), g2, dim3(P2_NT), 0, st, dz, g, w, dg, ws, T, d, bn);
    return check_launch("kdfm_dwconv_bwd_bn");
  }
  if (K == 31)
    hipLaunchKernelGGL((dwconv_bwd_kernel<31, true>), grid, dim3(256), 0, st, dz, g, w, dg, ws, T, d, (int)K, bn);
  else if (K == 9)
    hipLaunchKernelGGL((dwconv_bwd_kernel<9, true>), grid, dim3(256), 0, st, dz, g, w, dg, ws, T, d, (int)K, bn);
  else
    hipLaunchKernelGGL((dwconv_bwd_kernel<15, true>), grid, dim3(256), 0, st, dz, g, w, dg, ws, T, d, (int)K, bn);
  return check_launch("kdfm_dwconv_bwd_bn");
}

int kdfm_bn_silu_bwd_reduce(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                            const float* beta, double* red, int64_t rows, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dz && y && mean && rstd && gamma && beta && red, "null pointer");
  if (rows * d == 0) return KDFM_OK;
  int64_t gy = ceil_div(rows, 64);
  if (gy > 1024) gy = 1024;
  if (deterministic()) gy = 1;  // one workgroup per channel group: fixed summation order
  const int64_t rp = ceil_div(rows, gy);
  gy = ceil_div(rows, rp);
  hipLaunchKernelGGL(bn_silu_bwd_reduce_kernel, dim3((unsigned)ceil_div(d, 64), (unsigned)gy), dim3(256), 0,
                     as_stream(stream), dz, y, mean, rstd, gamma, beta, red, rows, d, rp);
  return check_launch("kdfm_bn_silu_bwd_reduce");
}

int kdfm_dwconv_bwd_fold(const float* ws, float* dw, float* db, int64_t B, int64_t T, int64_t d, int64_t K,
                         void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(ws && dw && db, "null pointer");
  const int64_t ld = d * (K + 1);
  // [dw | db] partial columns, one fold
  return launch_colsum2(ws, dw, d * K, db, B * ceil_div(T, TT), ld, ld, 1.f, as_stream(stream));
}

int kdfm_bn_finalize(const double* stats, const float* running_mean, const float* running_var, float* mean,
                     float* rstd, int64_t d, int64_t count, float eps, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(mean && rstd, "null pointer");
  KDFM_REQUIRE(stats || (running_mean && running_var), "need batch stats or running stats");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)ceil_div(d, 256)), dim3(256), 0, as_stream(stream), stats,
                     running_mean, running_var, mean, rstd, d, (double)count, eps);
  return check_launch("kdfm_bn_finalize");
}

int kdfm_bn_finalize_running(double* stats, float* running_mean, float* running_var, float* mean, float* rstd,
                             int64_t d, int64_t count, float eps, float momentum, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(stats && running_mean && running_var && mean && rstd, "null pointer");
  hipLaunchKernelGGL(bn_finalize_running_kernel, dim3((unsigned)ceil_div(d, 256)), dim3(256), 0, as_stream(stream),
                     stats, running_mean, running_var, mean, rstd, d, (double)count, eps, momentum);
  return check_launch("kdfm_bn_finalize_running");
}

int kdfm_bn_running_update(float* running_mean, float* running_var, const double* stats, int64_t d, int64_t count,
                           float momentum, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(running_mean && running_var && stats, "null pointer");
  hipLaunchKernelGGL(bn_running_kernel, dim3((unsigned)ceil_div(d, 256)), dim3(256), 0, as_stream(stream),
                     running_mean, running_var, stats, d, (double)count, momentum);
  return check_launch("kdfm_bn_running_update");
}

int kdfm_bn_silu_fwd(const float* y, const float* mean, const float* rstd, const float* gamma, const float* beta,
                     float* z, int64_t rows, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(y && mean && rstd && gamma && beta && z, "null pointer");
  const int64_t n = rows * d;
  if (n == 0) return KDFM_OK;
  if (ew4_ok(rows, d, {y, mean, rstd, gamma, beta, z})) {
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(bn_silu_fwd4_kernel<float>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), y,
                       mean, rstd, gamma, beta, z, (int)n4, (int)(d / 4));
    return check_launch("kdfm_bn_silu_fwd");
  }
  hipLaunchKernelGGL(bn_silu_fwd_kernel<float>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), y,
                     mean, rstd, gamma, beta, z, n, d);
  return check_launch("kdfm_bn_silu_fwd");
}

int kdfm_bn_silu_fwd_bf16(const float* y, const float* mean, const float* rstd, const float* gamma, const float* beta,
                          uint16_t* z, int64_t rows, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(y && mean && rstd && gamma && beta && z, "null pointer");
  const int64_t n = rows * d;
  if (n == 0) return KDFM_OK;
  if (ew4_ok(rows, d, {y, mean, rstd, gamma, beta, z})) {
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(bn_silu_fwd4_kernel<uint16_t>, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), y,
                       mean, rstd, gamma, beta, z, (int)n4, (int)(d / 4));
    return check_launch("kdfm_bn_silu_fwd");
  }
  hipLaunchKernelGGL(bn_silu_fwd_kernel<uint16_t>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream),
                     y, mean, rstd, gamma, beta, z, n, d);
  return check_launch("kdfm_bn_silu_fwd_bf16");
}

int kdfm_bn_silu_bwd2(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                      const float* beta, double* red_ws, double* red_next, float* dy, float* dgamma, float* dbeta,
                      int64_t rows, int64_t d, int32_t batch_stats, void* stream);

int kdfm_bn_silu_bwd(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, double* red_ws, float* dy, float* dgamma, float* dbeta, int64_t rows,
                     int64_t d, int32_t batch_stats, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(red_ws, "null pointer");
  if (rows * d == 0) return KDFM_OK;
  if (hipMemsetAsync(red_ws, 0, sizeof(double) * 2 * d, as_stream(stream)) != hipSuccess) {
    set_error("kdfm_bn_silu_bwd: memset failed");
    return KDFM_ELAUNCH;
  }
  return kdfm_bn_silu_bwd2(dz, y, mean, rstd, gamma, beta, red_ws, nullptr, dy, dgamma, dbeta, rows, d, batch_stats,
                           stream);
}

int kdfm_bn_silu_bwd2(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                      const float* beta, double* red_ws, double* red_next, float* dy, float* dgamma, float* dbeta,
                      int64_t rows, int64_t d, int32_t batch_stats, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dz && y && mean && rstd && gamma && beta && red_ws && dy && dgamma && dbeta, "null pointer");
  KDFM_REQUIRE(red_next != red_ws, "red_next must be another buffer");
  if (rows * d == 0) return KDFM_OK;
  hipStream_t st = as_stream(stream);
  // ~64 rows per workgroup: the per-channel f64 sums are latency-bound, so spread them wide
  int64_t gy = ceil_div(rows, 64);
  if (gy > 1024) gy = 1024;
  if (deterministic()) gy = 1;  // one workgroup per channel group: fixed summation order
  const int64_t rp = ceil_div(rows, gy);
  gy = ceil_div(rows, rp);
  hipLaunchKernelGGL(bn_silu_bwd_reduce_kernel, dim3((unsigned)ceil_div(d, 64), (unsigned)gy), dim3(256), 0, st, dz,
                     y, mean, rstd, gamma, beta, red_ws, rows, d, rp);
  int rc = check_launch("kdfm_bn_silu_bwd(reduce)");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_silu_bwd_apply_kernel, dim3((unsigned)ceil_div(rows * d, 256)), dim3(256), 0, st, dz, y, mean,
                     rstd, gamma, beta, red_ws, dy, dgamma, dbeta, rows * d, d, (double)rows, batch_stats, red_next);
  return check_launch("kdfm_bn_silu_bwd(apply)");
}

}  // extern "C"
