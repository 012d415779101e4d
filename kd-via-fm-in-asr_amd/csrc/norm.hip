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

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)) (+ dres)
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ g, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* dres,
                                                     float* dx, float* __restrict__ dg, float* __restrict__ db,
                                                     int64_t rows, int d, int64_t rows_per_block) {
  __shared__ float red_g[4][256];
  __shared__ float red_b[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float pg[MAXV], pb[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = (r0 + rows_per_block < rows) ? r0 + rows_per_block : rows;
  for (int64_t row = r0 + w; row < r1; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXV], gy[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < d) {
        const float dyv = dy[row * d + c];
        xh[i] = (x[row * d + c] - mu) * rs;
        gy[i] = dyv * g[c];
        pg[i] += dyv * xh[i];
        pb[i] += dyv;
      } else {
        xh[i] = 0.f;
        gy[i] = 0.f;
      }
      s1 += gy[i];
      s2 += gy[i] * xh[i];
    }
    s1 = wave_sum(s1) / d;
    s2 = wave_sum(s2) / d;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < d) {
        float v = rs * (gy[i] - s1 - xh[i] * s2);
        if (dres) v += dres[row * d + c];
        dx[row * d + c] = v;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < 256) {
      red_g[w][c] = pg[i];
      red_b[w][c] = pb[i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 256) {
    atomicAdd(dg + c, red_g[0][c] + red_g[1][c] + red_g[2][c] + red_g[3][c]);
    atomicAdd(db + c, red_b[0][c] + red_b[1][c] + red_b[2][c] + red_b[3][c]);
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

int kdfm_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                       const float* dres, float* dx, float* dgamma, float* dbeta, int64_t rows, int64_t d,
                       void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && x && gamma && mean && rstd && dx && dgamma && dbeta, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 256]");
  if (rows == 0) return KDFM_OK;
  int64_t blocks = ceil_div(rows, 32);
  if (blocks > 2048) blocks = 2048;
  const int64_t rpb = ceil_div(rows, blocks);
  blocks = ceil_div(rows, rpb);
  hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), dy, x, gamma, mean,
                     rstd, dres, dx, dgamma, dbeta, rows, (int)d, rpb);
  return check_launch("kdfm_layernorm_bwd");
}

}  // extern "C"
