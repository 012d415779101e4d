// LayerNorm forward/backward (Conformer pre-norms, NeMo ConformerLayer norm_* with eps 1e-5;
// called per layer from conformer_encoder.py:685-692).  One wave per row (d <= 256), fp32
// statistics; the backward fuses the residual-stream gradient add and reduces dgamma/dbeta with
// per-block partials + one atomic per column per block.
#include "common.h"

namespace kdfm {
namespace {

constexpr int MAXV = 4;  // d <= 256

__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                     const float* __restrict__ b, float* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int d, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * d;
  float v[MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < d) ? xr[c] : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    const float t = (c < d) ? v[i] - mu : 0.f;
    q += t * t;
  }
  const float rs = rsqrtf(wave_sum(q) / d + eps);
  float* yr = y + row * d;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < d) yr[c] = (v[i] - mu) * rs * g[c] + b[c];
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)) (+ dres).  Each block owns 64 rows
// (16 per wave, processed 4 at a time so their loads are in flight together) and writes its
// dgamma|dbeta column partials to part[block][2d]; the host folds them with launch_colsum.
template <int V>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ g, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* dres, float* dx,
                                                     float* __restrict__ part, int64_t rows, int d) {
  __shared__ float red[2][4][64 * V];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float gl[V], pg[V], pb[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = lane + 64 * i;
    gl[i] = (c < d) ? g[c] : 0.f;
    pg[i] = 0.f;
    pb[i] = 0.f;
  }
  const int64_t base = (int64_t)blockIdx.x * 64 + w * 16;
#pragma unroll 1
  for (int rb = 0; rb < 16; rb += 4) {
    float dyv[4][V], xv[4][V], mu[4], rs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = base + rb + j;
      const bool ok = row < rows;
      mu[j] = ok ? mean[row] : 0.f;
      rs[j] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        const bool in = ok && c < d;
        dyv[j][i] = in ? dy[row * d + c] : 0.f;
        xv[j][i] = in ? x[row * d + c] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = base + rb + j;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        const float xh = (c < d) ? (xv[j][i] - mu[j]) * rs[j] : 0.f;
        xv[j][i] = xh;
        const float gy = dyv[j][i] * gl[i];
        pg[i] += dyv[j][i] * xh;
        pb[i] += dyv[j][i];
        s1 += gy;
        s2 += gy * xh;
      }
      s1 = wave_sum(s1) / d;
      s2 = wave_sum(s2) / d;
      if (row < rows) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const int c = lane + 64 * i;
          if (c < d) {
            float v = rs[j] * (dyv[j][i] * gl[i] - s1 - xv[j][i] * s2);
            if (dres) v += dres[row * d + c];
            dx[row * d + c] = v;
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    red[0][w][lane + 64 * i] = pg[i];
    red[1][w][lane + 64 * i] = pb[i];
  }
  __syncthreads();
  float* pr = part + (int64_t)blockIdx.x * 2 * d;
  for (int c = threadIdx.x; c < d; c += 256) {
    pr[c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    pr[d + c] = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
  }
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd,
                       int64_t rows, int64_t d, float eps, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && gamma && beta && y && mean && rstd, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 256]");
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream), x, gamma,
                     beta, y, mean, rstd, rows, (int)d, eps);
  return check_launch("kdfm_layernorm_fwd");
}

int64_t kdfm_layernorm_bwd_ws(int64_t rows, int64_t d) { return kdfm::ceil_div(rows, 64) * 2 * d; }

int kdfm_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                       const float* dres, float* dx, float* dgamma, float* dbeta, float* ws, int64_t rows, int64_t d,
                       void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && x && gamma && mean && rstd && dx && dgamma && dbeta && ws, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 256]");
  if (rows == 0) return KDFM_OK;
  hipStream_t st = as_stream(stream);
  const int64_t blocks = ceil_div(rows, 64);
  const dim3 grid((unsigned)blocks), blk(256);
  switch ((d + 63) / 64) {
    case 1: hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, blk, 0, st, dy, x, gamma, mean, rstd, dres, dx, ws, rows, (int)d); break;
    case 2: hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, blk, 0, st, dy, x, gamma, mean, rstd, dres, dx, ws, rows, (int)d); break;
    case 3: hipLaunchKernelGGL(ln_bwd_kernel<3>, grid, blk, 0, st, dy, x, gamma, mean, rstd, dres, dx, ws, rows, (int)d); break;
    default: hipLaunchKernelGGL(ln_bwd_kernel<4>, grid, blk, 0, st, dy, x, gamma, mean, rstd, dres, dx, ws, rows, (int)d); break;
  }
  int rc = check_launch("kdfm_layernorm_bwd");
  if (rc) return rc;
  rc = launch_colsum(ws, dgamma, blocks, d, 2 * d, 1.f, st);
  if (rc) return rc;
  return launch_colsum(ws + d, dbeta, blocks, d, 2 * d, 1.f, st);
}

}  // extern "C"
