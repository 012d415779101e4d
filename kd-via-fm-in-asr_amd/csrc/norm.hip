// LayerNorm forward/backward (Conformer pre-norms, NeMo ConformerLayer norm_* with eps 1e-5;
// called per layer from conformer_encoder.py:685-692).  One wave per row (d <= 1024), fp32
// statistics; the backward fuses the residual-stream gradient add and reduces dgamma/dbeta with
// per-block partials folded in block order (one fold launch can serve several LayerNorms).
#include "common.h"

#include <initializer_list>

namespace kdfm {
namespace {

constexpr int MAXV = 16;  // d <= 1024 (FastConformer d_model 512 / 1024); V = 64-column groups per lane

template <int MAXV>
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

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)) (+ dres).  A block is 4 waves x LN_RPW
// rows (one row per wave per step, every load of the wave's rows issued before the first use), so a
// 12,832-row LayerNorm runs as ~800 workgroups: enough loads in flight to stream at HBM rate, where
// 64-row blocks (~200 workgroups) left most CUs idle.  The block's dgamma|dbeta column partials go
// to part[block][2d]; kdfm_ln_fold (one launch for several LayerNorms) sums them in block order.
constexpr int LN_RPW = 4;

// Wide rows (V > 4 column groups per lane, d > 256: Conformer-large / FastConformer-XL) keep one row's values at a
// time (3 V registers, the next row's loads issued before this row's reductions): holding all LN_RPW rows' dy, x and
// residual (12 V floats) spilled at d = 1024 (116 us per 6 432-row LayerNorm, profiles/r06/r6e).
template <int V>
// dy2 (nullable): a second gradient summed into dy on load (the encoder backward's layer-input gradient
// plus the hooked output's gradient, without an add launch in between)
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ g, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* dres, float* dx,
                                                     float* __restrict__ part, int64_t rows, int d,
                                                     const float* __restrict__ dy2) {
  __shared__ float red[2][4][64 * V];
  constexpr int RB = V > 4 ? 1 : LN_RPW;   // rows whose values are held at once
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float gl[V], pg[V], pb[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = lane + 64 * i;
    gl[i] = (c < d) ? g[c] : 0.f;
    pg[i] = 0.f;
    pb[i] = 0.f;
  }
  const int64_t base = ((int64_t)blockIdx.x * 4 + w) * LN_RPW;
#pragma unroll
  for (int j0 = 0; j0 < LN_RPW; j0 += RB) {
    float dyv[RB][V], xv[RB][V], rv[RB][V], mu[RB], rs[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int64_t row = base + j0 + j;
      const bool ok = row < rows;
      mu[j] = ok ? mean[row] : 0.f;
      rs[j] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        const bool in = ok && c < d;
        dyv[j][i] = in ? dy[row * d + c] + (dy2 ? dy2[row * d + c] : 0.f) : 0.f;
        xv[j][i] = in ? x[row * d + c] : 0.f;
        rv[j][i] = (in && dres) ? dres[row * d + c] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int64_t row = base + j0 + j;
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
          if (c < d) dx[row * d + c] = rs[j] * (dyv[j][i] * gl[i] - s1 - xv[j][i] * s2) + rv[j][i];
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

// Wide rows with d % 256 == 0 (Conformer-large 512, FastConformer-XL 1024): the same two kernels on 16-byte lanes --
// lane l owns columns 4 l + 256 i .. + 3 (NV = d / 256 float4 per row and tensor), so a row is NV 1 KB wave loads
// instead of 4 NV 256-byte ones.  Same arithmetic per element; the row sums group the columns per lane differently.
// BF: y is bf16 (round to nearest even -- the bits the large-tile GEMM's cast of an f32 y would produce), for an LN
// output whose every consumer reads bf16 operands (kdfm_layernorm_fwd_bf16)
template <int NV, bool BF = false>
__global__ __launch_bounds__(256) void ln_fwd_v4_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                        const float* __restrict__ b, void* __restrict__ yv,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                        int64_t rows, int d, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * d;
  float4 v[NV], gv[NV], bv[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    v[i] = *reinterpret_cast<const float4*>(xr + c);
    gv[i] = *reinterpret_cast<const float4*>(g + c);
    bv[i] = *reinterpret_cast<const float4*>(b + c);
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mu = wave_sum(s) / d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float a0 = v[i].x - mu, a1 = v[i].y - mu, a2 = v[i].z - mu, a3 = v[i].w - mu;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const float rs = rsqrtf(wave_sum(q) / d + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * lane + 256 * i;
    float4 o;
    o.x = (v[i].x - mu) * rs * gv[i].x + bv[i].x;
    o.y = (v[i].y - mu) * rs * gv[i].y + bv[i].y;
    o.z = (v[i].z - mu) * rs * gv[i].z + bv[i].z;
    o.w = (v[i].w - mu) * rs * gv[i].w + bv[i].w;
    if constexpr (BF)
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(yv) + row * d + c) =
          make_uint2(pack_bf16x2(o.x, o.y), pack_bf16x2(o.z, o.w));
    else
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(yv) + row * d + c) = o;
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

// rows per wave of the 16-byte-lane backward: one -- 6 432-row LayerNorms then run as 1 608 workgroups (4 rows
// each) instead of 402 (1.6 waves per SIMD at 221 registers: latency-bound, 62 us in the XL step), at four times the
// dgamma / dbeta partial rows (ln_rows_per_block)
constexpr int LN_RPW_V4 = 1;

template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_v4_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                        const float* __restrict__ g, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, const float* dres, float* dx,
                                                        float* __restrict__ part, int64_t rows, int d,
                                                        const float* __restrict__ dy2) {
  __shared__ float red[2][4][256 * NV];
  constexpr int RPW = LN_RPW_V4;
  constexpr int RB = RPW;   // rows whose values are held at once
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float gl[NV][4], pg[NV][4], pb[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float4 t = *reinterpret_cast<const float4*>(g + 4 * lane + 256 * i);
    gl[i][0] = t.x; gl[i][1] = t.y; gl[i][2] = t.z; gl[i][3] = t.w;
#pragma unroll
    for (int e = 0; e < 4; ++e) pg[i][e] = pb[i][e] = 0.f;
  }
  const int64_t base = ((int64_t)blockIdx.x * 4 + w) * RPW;
#pragma unroll
  for (int j0 = 0; j0 < RPW; j0 += RB) {
    float dyv[RB][NV][4], xv[RB][NV][4], rv[RB][NV][4], mu[RB], rs[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int64_t row = base + j0 + j;
      const bool ok = row < rows;
      const int64_t r = ok ? row : 0;
      mu[j] = mean[r];
      rs[j] = rstd[r];
      const float m = ok ? 1.f : 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int64_t o = r * d + 4 * lane + 256 * i;
        float4 a = *reinterpret_cast<const float4*>(dy + o);
        if (dy2) {
          const float4 a2 = *reinterpret_cast<const float4*>(dy2 + o);
          a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
        }
        const float4 xx = *reinterpret_cast<const float4*>(x + o);
        const float4 rr = dres ? *reinterpret_cast<const float4*>(dres + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        dyv[j][i][0] = a.x * m; dyv[j][i][1] = a.y * m; dyv[j][i][2] = a.z * m; dyv[j][i][3] = a.w * m;
        xv[j][i][0] = xx.x; xv[j][i][1] = xx.y; xv[j][i][2] = xx.z; xv[j][i][3] = xx.w;
        rv[j][i][0] = rr.x; rv[j][i][1] = rr.y; rv[j][i][2] = rr.z; rv[j][i][3] = rr.w;
      }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int64_t row = base + j0 + j;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[j][i][e] - mu[j]) * rs[j];
          xv[j][i][e] = xh;
          const float gy = dyv[j][i][e] * gl[i][e];
          pg[i][e] += dyv[j][i][e] * xh;
          pb[i][e] += dyv[j][i][e];
          s1 += gy;
          s2 += gy * xh;
        }
      s1 = wave_sum(s1) / d;
      s2 = wave_sum(s2) / d;
      if (row < rows) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = rs[j] * (dyv[j][i][e] * gl[i][e] - s1 - xv[j][i][e] * s2) + rv[j][i][e];
          *reinterpret_cast<float4*>(dx + row * d + 4 * lane + 256 * i) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    *reinterpret_cast<float4*>(&red[0][w][4 * lane + 256 * i]) = make_float4(pg[i][0], pg[i][1], pg[i][2], pg[i][3]);
    *reinterpret_cast<float4*>(&red[1][w][4 * lane + 256 * i]) = make_float4(pb[i][0], pb[i][1], pb[i][2], pb[i][3]);
  }
  __syncthreads();
  float* pr = part + (int64_t)blockIdx.x * 2 * d;
  for (int c = threadIdx.x; c < d; c += 256) {
    pr[c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    pr[d + c] = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
  }
}

__host__ inline bool ln_v4_ok(int64_t d, std::initializer_list<const void*> ptrs) {
  if (d % 256 != 0 || d > 1024) return false;
  for (const void* p : ptrs)
    if (((uintptr_t)p) & 15) return false;
  return true;
}

// rows per dgamma / dbeta partial row of the backward (the workspace and the fold follow it): 4 waves x LN_RPW rows,
// or 4 x LN_RPW_V4 on the 16-byte-lane path (d % 256 == 0, which then requires 16-byte aligned operands)
__host__ inline int64_t ln_rows_per_block(int64_t d) {
  return (d % 256 == 0 && d <= 1024) ? 4 * LN_RPW_V4 : 4 * LN_RPW;
}

// Ordered fold of LayerNorm partials for up to KDFM_LN_FOLD_MAX LayerNorms in one launch:
// dgamma_e[c] += sum_b part_e[b][c], dbeta_e[c] += sum_b part_e[b][d + c].  grid = (column groups of
// 64 over 2d, entries); lane = column, the 4 waves stride the partial rows, fixed-order combine
// (deterministic: one workgroup owns each output column).
struct LnFold {
  const float* part[KDFM_LN_FOLD_MAX];
  float* dg[KDFM_LN_FOLD_MAX];
  float* db[KDFM_LN_FOLD_MAX];
};

// 16 waves per block, lane = output column: wave w sums the parts b = w, w + 16, ... with four
// independent accumulators (many loads in flight; the 4-wave version was latency-bound at ~50 us per
// layer), then a fixed-order combine in LDS — the same order every run (deterministic).
constexpr int LNF_WAVES = 16;

__global__ __launch_bounds__(64 * LNF_WAVES) void ln_fold_kernel(LnFold f, int64_t nparts, int d) {
  __shared__ float red[LNF_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.y;
  const int c = blockIdx.x * 64 + lane;
  const float* part = f.part[e];
  const int64_t ld = 2 * (int64_t)d;
  // eight independent accumulators (eight loads in flight per lane; four left the 16-wave fold latency-bound at
  // ~12 us for a layer's six 802-row partial sets), combined in a fixed order
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < 2 * d) {
    int64_t b = w;
    for (; b + 7 * LNF_WAVES < nparts; b += 8 * LNF_WAVES) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(b + u * LNF_WAVES) * ld + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += v[u];
    }
    for (; b < nparts; b += LNF_WAVES) s[0] += part[b * ld + c];
  }
  red[w][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (w == 0 && c < 2 * d) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < LNF_WAVES; ++i) v += red[i][lane];
    if (c < d)
      f.dg[e][c] += v;
    else
      f.db[e][c - d] += v;
  }
}

int ln_fold(const float* const* parts, float* const* dgs, float* const* dbs, int n, int64_t nparts, int64_t d,
            hipStream_t st) {
  LnFold f{};
  for (int i = 0; i < n; ++i) {
    f.part[i] = parts[i];
    f.dg[i] = dgs[i];
    f.db[i] = dbs[i];
  }
  hipLaunchKernelGGL(ln_fold_kernel, dim3((unsigned)ceil_div(2 * d, 64), (unsigned)n), dim3(64 * LNF_WAVES), 0, st, f,
                     nparts, (int)d);
  return check_launch("kdfm_ln_fold");
}

int ln_bwd_launch(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                  const float* dres, float* dx, float* part, int64_t rows, int64_t d, hipStream_t st,
                  const float* dy2 = nullptr) {
  const int64_t blocks = ceil_div(rows, ln_rows_per_block(d));
  const dim3 grid((unsigned)blocks), blk(256);
  if (d % 256 == 0 && d <= 1024) {
    KDFM_REQUIRE(ln_v4_ok(d, {dy, x, gamma, dres, dx, dy2}), "d % 256 == 0: 16-byte aligned operands");
#define LNB4(NV) hipLaunchKernelGGL(ln_bwd_v4_kernel<NV>, grid, blk, 0, st, dy, x, gamma, mean, rstd, dres, dx, part, rows, (int)d, dy2)
    if (d == 256) LNB4(1);
    else if (d == 512) LNB4(2);
    else if (d == 768) LNB4(3);
    else LNB4(4);
#undef LNB4
    return check_launch("kdfm_layernorm_bwd");
  }
  const int64_t v = (d + 63) / 64;
#define LNB(V) hipLaunchKernelGGL(ln_bwd_kernel<V>, grid, blk, 0, st, dy, x, gamma, mean, rstd, dres, dx, part, rows, (int)d, dy2)
  if (v == 1) LNB(1);
  else if (v == 2) LNB(2);
  else if (v == 3) LNB(3);
  else if (v == 4) LNB(4);
  else if (v <= 8) LNB(8);
  else LNB(16);
#undef LNB
  return check_launch("kdfm_layernorm_bwd");
}

int ln_fwd_launch(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd,
                  int64_t rows, int64_t d, float eps, hipStream_t st) {
  const dim3 grid((unsigned)ceil_div(rows, 4)), blk(256);
  if (ln_v4_ok(d, {x, gamma, beta, y})) {
#define LNF4(NV) hipLaunchKernelGGL((ln_fwd_v4_kernel<NV, false>), grid, blk, 0, st, x, gamma, beta, (void*)y, mean, rstd, rows, (int)d, eps)
    if (d == 256) LNF4(1);
    else if (d == 512) LNF4(2);
    else if (d == 768) LNF4(3);
    else LNF4(4);
#undef LNF4
    return check_launch("kdfm_layernorm_fwd");
  }
  const int64_t v = (d + 63) / 64;
#define LNF(V) hipLaunchKernelGGL(ln_fwd_kernel<V>, grid, blk, 0, st, x, gamma, beta, y, mean, rstd, rows, (int)d, eps)
  if (v == 1) LNF(1);
  else if (v == 2) LNF(2);
  else if (v == 3) LNF(3);
  else if (v == 4) LNF(4);
  else if (v <= 8) LNF(8);
  else LNF(16);
#undef LNF
  return check_launch("kdfm_layernorm_fwd");
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd,
                       int64_t rows, int64_t d, float eps, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && gamma && beta && y && mean && rstd, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 1024]");
  if (rows == 0) return KDFM_OK;
  return ln_fwd_launch(x, gamma, beta, y, mean, rstd, rows, d, eps, as_stream(stream));
}

int kdfm_layernorm_fwd_bf16(const float* x, const float* gamma, const float* beta, uint16_t* y, float* mean,
                            float* rstd, int64_t rows, int64_t d, float eps, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && gamma && beta && y && mean && rstd, "null pointer");
  KDFM_REQUIRE(ln_v4_ok(d, {x, gamma, beta, y}), "d % 256 == 0, d <= 1024, 16-byte aligned rows");
  if (rows == 0) return KDFM_OK;
  const dim3 grid((unsigned)ceil_div(rows, 4)), blk(256);
  hipStream_t st = as_stream(stream);
#define LNF4B(NV) hipLaunchKernelGGL((ln_fwd_v4_kernel<NV, true>), grid, blk, 0, st, x, gamma, beta, (void*)y, mean, rstd, rows, (int)d, eps)
  if (d == 256) LNF4B(1);
  else if (d == 512) LNF4B(2);
  else if (d == 768) LNF4B(3);
  else LNF4B(4);
#undef LNF4B
  return check_launch("kdfm_layernorm_fwd_bf16");
}

int64_t kdfm_layernorm_bwd_ws(int64_t rows, int64_t d) { return kdfm::ceil_div(rows, kdfm::ln_rows_per_block(d)) * 2 * d; }

int kdfm_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                       const float* dres, float* dx, float* dgamma, float* dbeta, float* ws, int64_t rows, int64_t d,
                       void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && x && gamma && mean && rstd && dx && dgamma && dbeta && ws, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 1024]");
  if (rows == 0) return KDFM_OK;
  hipStream_t st = as_stream(stream);
  int rc = ln_bwd_launch(dy, x, gamma, mean, rstd, dres, dx, ws, rows, d, st);
  if (rc) return rc;
  const float* parts[1] = {ws};
  float* dgs[1] = {dgamma};
  float* dbs[1] = {dbeta};
  return ln_fold(parts, dgs, dbs, 1, ceil_div(rows, ln_rows_per_block(d)), d, st);
}

int kdfm_layernorm_bwd_part(const float* dy, const float* x, const float* gamma, const float* mean,
                            const float* rstd, const float* dres, float* dx, float* part, int64_t rows, int64_t d,
                            void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && x && gamma && mean && rstd && dx && part, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 1024]");
  if (rows == 0) return KDFM_OK;
  return ln_bwd_launch(dy, x, gamma, mean, rstd, dres, dx, part, rows, d, as_stream(stream));
}

int kdfm_layernorm_bwd_part2(const float* dy, const float* dy2, const float* x, const float* gamma, const float* mean,
                             const float* rstd, const float* dres, float* dx, float* part, int64_t rows, int64_t d,
                             void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && dy2 && x && gamma && mean && rstd && dx && part, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 64 * MAXV, "d must be in (0, 1024]");
  if (rows == 0) return KDFM_OK;
  return ln_bwd_launch(dy, x, gamma, mean, rstd, dres, dx, part, rows, d, as_stream(stream), dy2);
}

int kdfm_ln_fold(const float* const* parts, float* const* dgamma, float* const* dbeta, int32_t n, int64_t rows,
                 int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(parts && dgamma && dbeta && n >= 1 && n <= KDFM_LN_FOLD_MAX, "1..KDFM_LN_FOLD_MAX LayerNorms");
  for (int i = 0; i < n; ++i) KDFM_REQUIRE(parts[i] && dgamma[i] && dbeta[i], "null pointer");
  if (rows == 0) return KDFM_OK;
  return ln_fold(parts, dgamma, dbeta, n, ceil_div(rows, ln_rows_per_block(d)), d, as_stream(stream));
}

}  // extern "C"
