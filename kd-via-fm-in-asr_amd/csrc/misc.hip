// Memory-bound glue of the step: fills, strided axpby, dropout application, the attention
// q+u / q+v prep, conv-weight re-layouts, and the ver5 KD-head pieces that are not GEMMs:
// NoiseAdapter gating (asr_train_diffm.py:425-442) and the FlowMatchingModule time embedding
// (asr_train_diffm.py:1368-1378: Linear(1->32) of t = i/steps, concatenated to the 96-d state;
// folded here into a per-step bias of the first meta-encoder Linear).
#include "common.h"

namespace kdfm {
namespace {

__global__ __launch_bounds__(256) void fill_kernel(float* x, float v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = v;
}

// out[r,c] = alpha*a[r,c] + beta*b[r,c]
__global__ __launch_bounds__(256) void axpby_kernel(const float* a, int64_t lda, const float* b, int64_t ldb, float* out,
                                                    int64_t ldo, int64_t rows, int64_t cols, float alpha, float beta) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols, c = i - r * cols;
  float v = alpha * a[r * lda + c];
  if (b) v += beta * b[r * ldb + c];
  out[r * ldo + c] = v;
}

// out[r, c] = x[r, c] * s[r / rows_per_s] * alpha   (device-scalar scaling, no host sync)
__global__ __launch_bounds__(256) void rowscale_kernel(const float* x, float* out, int64_t rows, int64_t cols,
                                                       const float* s, int64_t rows_per_s, float alpha) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols;
  out[i] = x[i] * s[r / rows_per_s] * alpha;
}

// out = (y > 0) ? dy : 0   (ReLU backward from the saved activation)
__global__ __launch_bounds__(256) void relu_mask_kernel(const float* dy, const float* y, float* out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (y[i] > 0.f) ? dy[i] : 0.f;
}

// loss_acc[0] += scale * sum (a - b)^2 ; grad (optional) = gscale * (a - b)
__global__ __launch_bounds__(256) void mse_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                  float* __restrict__ grad, float* __restrict__ loss_acc, int64_t n,
                                                  float scale, float gscale) {
  __shared__ float red[4];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float part = 0.f;
  if (i < n) {
    const float d = a[i] - b[i];
    part = d * d;
    if (grad) grad[i] = gscale * d;
  }
  part = wave_sum(part);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss_acc, scale * (red[0] + red[1] + red[2] + red[3]));
}

// nn.L1Loss pieces (kd_crit with kd_loss_type="l1", asr_train_diffm.py:557): |a-b| summed, torch's
// sign(a-b) subgradient (0 at a == b)
__global__ __launch_bounds__(256) void l1_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                 float* __restrict__ grad, float* __restrict__ loss_acc, int64_t n,
                                                 float scale, float gscale) {
  __shared__ float red[4];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float part = 0.f;
  if (i < n) {
    const float d = a[i] - b[i];
    part = fabsf(d);
    if (grad) grad[i] = d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f);
  }
  part = wave_sum(part);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss_acc, scale * (red[0] + red[1] + red[2] + red[3]));
}

// out = scale * dropout(x) with the flat-index mask of the GEMM epilogue (idx = r*cols + c)
// O = uint16_t: the result rounded to bf16 (kdfm_dropout_bf16: an operand only bf16-operand products read)
template <typename O>
__global__ __launch_bounds__(256) void dropout_kernel(const float* x, O* out, int64_t n, float p, float scale,
                                                      const uint64_t* seed_ptr, uint64_t st) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = x[i] * scale;
  if (p > 0.f) v = dropout_keep(load_seed(seed_ptr), st, (uint64_t)i, p) ? v / (1.f - p) : 0.f;
  if constexpr (sizeof(O) == 2)
    out[i] = f2bf(v);
  else
    out[i] = v;
}

// 16-byte lanes, 32-bit index math (FastConformer-XL: the 64-bit division per element made the 6 432 x 1024 pass
// take 37 us): thread = 4 consecutive columns of one row
__global__ __launch_bounds__(256) void qkv_prep4_kernel(const float* __restrict__ qkv, const float* __restrict__ u,
                                                        const float* __restrict__ v, float* __restrict__ qu,
                                                        float* __restrict__ qv, int n4, int d4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int r = i / d4, j = i - r * d4;
  const float4 q = reinterpret_cast<const float4*>(qkv)[(int64_t)r * 3 * d4 + j];
  const float4 a = reinterpret_cast<const float4*>(u)[j], b = reinterpret_cast<const float4*>(v)[j];
  reinterpret_cast<float4*>(qu)[i] = make_float4(q.x + a.x, q.y + a.y, q.z + a.z, q.w + a.w);
  reinterpret_cast<float4*>(qv)[i] = make_float4(q.x + b.x, q.y + b.y, q.z + b.z, q.w + b.w);
}

// 4 consecutive elements per thread (16-byte loads, aligned buffers): the same per-element mask and scaling
template <typename O>
__global__ __launch_bounds__(256) void dropout4_kernel(const float* x, O* out, int64_t n4, float p, float scale,
                                                       const uint64_t* seed_ptr, uint64_t st) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= n4) return;
  const float4 xv = reinterpret_cast<const float4*>(x)[q];
  float v[4] = {xv.x * scale, xv.y * scale, xv.z * scale, xv.w * scale};
  if (p > 0.f) {
    const uint64_t sd = load_seed(seed_ptr);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = dropout_keep(sd, st, (uint64_t)(4 * q + e), p) ? v[e] / (1.f - p) : 0.f;
  }
  if constexpr (sizeof(O) == 2)
    reinterpret_cast<uint2*>(out)[q] = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  else
    reinterpret_cast<float4*>(out)[q] = make_float4(v[0], v[1], v[2], v[3]);
}

// qu[r, j] = qkv[r, j] + u[j]; qv[r, j] = qkv[r, j] + v[j]   (j = h*dk + c over d columns)
__global__ __launch_bounds__(256) void qkv_prep_kernel(const float* __restrict__ qkv, const float* __restrict__ u,
                                                       const float* __restrict__ v, float* __restrict__ qu,
                                                       float* __restrict__ qv, int64_t rows, int64_t d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * d) return;
  const int64_t r = i / d, j = i - r * d;
  const float q = qkv[r * 3 * d + j];
  qu[i] = q + u[j];
  qv[i] = q + v[j];
}

// NeMo Conv1d weight (O, I, K) -> GEMM layouts: fwd[o][k][i] = W[o][i][k];
// bwd (transposed + flipped taps) [i][k][o] = W[o][i][K-1-k]
__global__ __launch_bounds__(256) void convw_prep_kernel(const float* __restrict__ W, float* __restrict__ fwd,
                                                         float* __restrict__ bwd, int64_t O, int64_t I, int64_t K) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= O * I * K) return;
  const int64_t k = idx % K, i = (idx / K) % I, o = idx / (K * I);
  const float w = W[idx];
  if (fwd) fwd[(o * K + k) * I + i] = w;
  if (bwd) bwd[(i * K + (K - 1 - k)) * O + o] = w;
}

// dW[o][i][k] += alpha * G[o][k][i]
__global__ __launch_bounds__(256) void convw_grad_kernel(const float* __restrict__ G, float* __restrict__ dW, int64_t O,
                                                         int64_t I, int64_t K, float alpha) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= O * I * K) return;
  const int64_t k = idx % K, i = (idx / K) % I, o = idx / (K * I);
  dW[idx] += alpha * G[(o * K + k) * I + i];
}

// NoiseAdapter: gamma = sigmoid(h . w2 + b2); zn = gamma*zs + (1-gamma)*eps   (one wave per row)
__global__ __launch_bounds__(256) void adapter_fwd_kernel(const float* __restrict__ zs, const float* __restrict__ h,
                                                          const float* __restrict__ w2, const float* __restrict__ b2,
                                                          const float* __restrict__ eps_in, float* __restrict__ zn,
                                                          float* __restrict__ gamma, int64_t rows, int L,
                                                          const uint64_t* seed_ptr, uint64_t st) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float s = 0.f;
  for (int c = lane; c < L; c += 64) s += h[r * L + c] * w2[c];
  s = wave_sum(s) + b2[0];
  const float g = sigmoidf_(s);
  const uint64_t seed = eps_in ? 0 : load_seed(seed_ptr);
  for (int c = lane; c < L; c += 64) {
    const float e = eps_in ? eps_in[r * L + c] : rng_normal(seed, st, (uint64_t)(r * L + c));
    zn[r * L + c] = g * zs[r * L + c] + (1.f - g) * e;
  }
  if (lane == 0) gamma[r] = g;
}

// the same with 16 lanes per row (L a multiple of 16): a wave has 4 rows' loads in flight instead of
// one row's dependent reduce-then-mix chain (205k rows of 96 at the bench shape)
template <int PL>
__global__ __launch_bounds__(256) void adapter_fwd16_kernel(const float* __restrict__ zs, const float* __restrict__ h,
                                                            const float* __restrict__ w2, const float* __restrict__ b2,
                                                            const float* __restrict__ eps_in, float* __restrict__ zn,
                                                            float* __restrict__ gamma, int64_t rows, int L,
                                                            const uint64_t* seed_ptr, uint64_t st) {
  const int sub = threadIdx.x & 15;
  const uint64_t seed = eps_in ? 0 : load_seed(seed_ptr);
  float w2v[PL];
#pragma unroll
  for (int k = 0; k < PL; ++k) w2v[k] = w2[sub + 16 * k];
  const float bias = b2[0];
  for (int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); r < rows; r += (int64_t)gridDim.x * 16) {
    float hv[PL], z[PL], e[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int64_t off = r * L + sub + 16 * k;
      hv[k] = h[off];
      z[k] = zs[off];
      e[k] = eps_in ? eps_in[off] : rng_normal(seed, st, (uint64_t)off);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PL; ++k) s += hv[k] * w2v[k];
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 16);
    const float g = sigmoidf_(s + bias);
#pragma unroll
    for (int k = 0; k < PL; ++k) zn[r * L + sub + 16 * k] = g * z[k] + (1.f - g) * e[k];
    if (sub == 0) gamma[r] = g;
  }
}

// backward: dzs = g*dzn ; dgl = g(1-g) * sum_c dzn*(zs-eps) ; dh = dgl*w2*(h>0) ; dw2 += dgl*h ; db2 += dgl.
// 16 lanes per row (lane k of the group owns columns k, k+16, ..: 64-byte coalesced segments), 4 rows per
// wave and 16 per workgroup in flight, so a row's loads overlap the others' instead of one dependent
// chain per row; each workgroup writes its (dw2 | db2) partial to ws, folded in workgroup order by
// adapter_bwd_fold_kernel (deterministic in either reduction mode, no atomics)
constexpr int AB_MAXPL = 8;   // L <= 128
template <int PL>
__global__ __launch_bounds__(256) void adapter_bwd_kernel(const float* __restrict__ dzn, const float* __restrict__ zs,
                                                          const float* __restrict__ h, const float* __restrict__ gamma,
                                                          const float* __restrict__ w2, const float* __restrict__ eps_in,
                                                          float* __restrict__ dzs, float* __restrict__ dh,
                                                          float* __restrict__ part, int64_t rows, int L,
                                                          const uint64_t* seed_ptr, uint64_t st, int64_t rows_per) {
  __shared__ float red[16][AB_MAXPL * 16 + 1];
  const int sub = threadIdx.x & 15, grp = threadIdx.x >> 4;   // 16 row groups of 16 lanes
  const uint64_t seed = eps_in ? 0 : load_seed(seed_ptr);
  float pw[PL], pb = 0.f, w2v[PL];
#pragma unroll
  for (int k = 0; k < PL; ++k) {
    pw[k] = 0.f;
    w2v[k] = w2[sub + 16 * k];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per;
  const int64_t r1 = (r0 + rows_per < rows) ? r0 + rows_per : rows;
  for (int64_t r = r0 + grp; r < r1; r += 16) {
    const float g = gamma[r];
    float d[PL], z[PL], hv[PL], e[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int64_t off = r * L + sub + 16 * k;
      d[k] = dzn[off];
      z[k] = zs[off];
      hv[k] = h[off];
      e[k] = eps_in ? eps_in[off] : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int64_t off = r * L + sub + 16 * k;
      const float ev = eps_in ? e[k] : rng_normal(seed, st, (uint64_t)off);
      s += d[k] * (z[k] - ev);
      dzs[off] = g * d[k];
    }
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 16);
    const float dgl = s * g * (1.f - g);
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      dh[r * L + sub + 16 * k] = (hv[k] > 0.f) ? dgl * w2v[k] : 0.f;
      pw[k] += dgl * hv[k];
    }
    pb += dgl;
  }
#pragma unroll
  for (int k = 0; k < PL; ++k) red[grp][sub + 16 * k] = pw[k];
  if (sub == 0) red[grp][AB_MAXPL * 16] = pb;
  __syncthreads();
  // this workgroup's partial: column c summed over the 16 row groups in order
  for (int c = threadIdx.x; c <= L; c += 256) {
    const int cc = c < L ? c : AB_MAXPL * 16;
    float a = 0.f;
    for (int q = 0; q < 16; ++q) a += red[q][cc];
    part[(int64_t)blockIdx.x * (L + 1) + c] = a;
  }
}

// dw2[c] += sum_b part[b][c] (c < L), db2 += sum_b part[b][L]: one workgroup per column, fixed order
__global__ __launch_bounds__(256) void adapter_bwd_fold_kernel(const float* __restrict__ part, int64_t nb, int L,
                                                               float* __restrict__ dw2, float* __restrict__ db2) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float a = 0.f;
  for (int64_t b = threadIdx.x; b < nb; b += 256) a += part[b * (L + 1) + c];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (c < L) dw2[c] += red[0];
    else db2[0] += red[0];
  }
}

constexpr int64_t AB_BLOCKS = 2048;

// per FM step j (t = (S-j)/S): e_j = w_te*t + b_te ; c_j = W1[:, L:] e_j + b1   (W1 is L x (L+E))
__global__ __launch_bounds__(256) void fm_step_bias_kernel(const float* __restrict__ w_te, const float* __restrict__ b_te,
                                                           const float* __restrict__ W1, const float* __restrict__ b1,
                                                           float* __restrict__ cvec, float* __restrict__ evec, int L,
                                                           int E, int S) {
  const int j = blockIdx.x;
  const float t = (float)(S - j) / (float)S;
  for (int o = threadIdx.x; o < L; o += 256) {
    float acc = b1[o];
    for (int q = 0; q < E; ++q) acc += W1[o * (L + E) + L + q] * (w_te[q] * t + b_te[q]);
    cvec[j * L + o] = acc;
  }
  for (int q = threadIdx.x; q < E; q += 256) evec[j * E + q] = w_te[q] * t + b_te[q];
}

// given dc_j (S x L): dW1[:, L:] += dc_j e_j^T ; db1 += dc_j ; de_j = W1[:, L:]^T dc_j ;
// dw_te += de_j * t_j ; db_te += de_j.  Workgroup q < E owns time-embedding feature q (thread o = output
// row o: its dW1 entry, and w_o * sum_j t_j dc_j[o] / w_o * sum_j dc_j[o] tree-reduced over o in a fixed
// order); workgroup E sums db1.  (One workgroup looping 8 x L serial loads per feature took 280 us.)
__global__ __launch_bounds__(256) void fm_time_bwd_kernel(const float* __restrict__ dc, const float* __restrict__ evec,
                                                          const float* __restrict__ W1, float* __restrict__ dW1,
                                                          float* __restrict__ db1, float* __restrict__ dw_te,
                                                          float* __restrict__ db_te, int L, int E, int S) {
  __shared__ float rw[256], rb[256];
  const int q = blockIdx.x, o = threadIdx.x;
  if (q == E) {
    if (o < L) {
      float acc = 0.f;
      for (int j = 0; j < S; ++j) acc += dc[j * L + o];
      db1[o] += acc;
    }
    return;
  }
  float gw = 0.f, gb = 0.f;
  if (o < L) {
    float dw = 0.f, st = 0.f, s1 = 0.f;
    for (int j = 0; j < S; ++j) {
      const float d = dc[j * L + o];
      dw += d * evec[j * E + q];
      st += d * ((float)(S - j) / (float)S);
      s1 += d;
    }
    const int64_t wi = (int64_t)o * (L + E) + L + q;
    dW1[wi] += dw;
    const float w = W1[wi];
    gw = w * st;
    gb = w * s1;
  }
  rw[o] = gw;
  rb[o] = gb;
  __syncthreads();
  for (int h = 128; h >= 1; h >>= 1) {
    if (o < h) {
      rw[o] += rw[o + h];
      rb[o] += rb[o + h];
    }
    __syncthreads();
  }
  if (o == 0) {
    dw_te[q] += rw[0];
    db_te[q] += rb[0];
  }
}

// sinusoidal relative position table, positions T-1 ... -(T-1) (RelPositionalEncoding, A.4)
__global__ __launch_bounds__(256) void relpos_table_kernel(float* __restrict__ pe, int64_t T, int64_t d) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (2 * T - 1) * d) return;
  const int64_t p = idx / d, c = idx % d;
  const double pos = (double)(T - 1 - p);
  const int64_t i2 = c & ~1ll;
  const double div = exp((double)i2 * -(log(10000.0) / (double)d));
  pe[idx] = (float)((c & 1) ? cos(pos * div) : sin(pos * div));
}

// mel_len = L // hop (pinned: frames - 1); two striding convs: floor((l - 1)/2 + 1)
__global__ void lengths_kernel(const int64_t* __restrict__ wl, int64_t* __restrict__ ml, int64_t* __restrict__ l1,
                               int64_t* __restrict__ l2, int64_t B, int64_t hop) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const int64_t m = wl[b] / hop;
  const int64_t a = (int64_t)floor(((double)m - 1.0) / 2.0 + 1.0);
  const int64_t c = (int64_t)floor(((double)a - 1.0) / 2.0 + 1.0);
  ml[b] = m;
  if (l1) l1[b] = a;
  if (l2) l2[b] = c;
}

// step counter / per-step RNG seed advance (graph-replay safe: runs on device)
__global__ void step_advance_kernel(int64_t* step, uint64_t* seed) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (step) step[0] += 1;
    if (seed) seed[0] = mix64(seed[0] + 0x632BE59BD9B4E019ull);
  }
}

}  // namespace
}  // namespace kdfm

extern "C" {

#define KDFM_1D(kernel, n, ...)                                                                              \
  do {                                                                                                       \
    if ((n) == 0) return KDFM_OK;                                                                            \
    hipLaunchKernelGGL(kernel, dim3((unsigned)kdfm::ceil_div((n), 256)), dim3(256), 0,                        \
                       kdfm::as_stream(stream), __VA_ARGS__);                                                \
  } while (0)

int kdfm_fill(float* x, float value, int64_t n, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x || n == 0, "null pointer");
  KDFM_1D(fill_kernel, n, x, value, n);
  return check_launch("kdfm_fill");
}

int kdfm_axpby(const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int64_t ldo, int64_t rows,
               int64_t cols, float alpha, float beta, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(a && out, "null pointer");
  KDFM_1D(axpby_kernel, rows * cols, a, lda, b, ldb, out, ldo, rows, cols, alpha, beta);
  return check_launch("kdfm_axpby");
}

int kdfm_dropout(const float* x, float* out, int64_t n, float p, float scale, const uint64_t* seed,
                 uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && out, "null pointer");
  KDFM_REQUIRE(p >= 0.f && p < 1.f && (p == 0.f || seed), "dropout p / seed");
  if (n % 4 == 0 && ((((uintptr_t)x) | ((uintptr_t)out)) & 15) == 0) {
    hipLaunchKernelGGL(dropout4_kernel<float>, dim3((unsigned)ceil_div(n / 4, 256)), dim3(256), 0, as_stream(stream), x,
                       out, n / 4, p, scale, seed, rng_stream);
    return check_launch("kdfm_dropout");
  }
  KDFM_1D(dropout_kernel<float>, n, x, out, n, p, scale, seed, rng_stream);
  return check_launch("kdfm_dropout");
}

int kdfm_dropout_bf16(const float* x, uint16_t* out, int64_t n, float p, float scale, const uint64_t* seed,
                      uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && out, "null pointer");
  KDFM_REQUIRE(p >= 0.f && p < 1.f && (p == 0.f || seed), "dropout p / seed");
  if (n % 4 == 0 && (((uintptr_t)x) & 15) == 0 && (((uintptr_t)out) & 7) == 0) {
    hipLaunchKernelGGL(dropout4_kernel<uint16_t>, dim3((unsigned)ceil_div(n / 4, 256)), dim3(256), 0, as_stream(stream), x,
                       out, n / 4, p, scale, seed, rng_stream);
    return check_launch("kdfm_dropout_bf16");
  }
  KDFM_1D(dropout_kernel<uint16_t>, n, x, out, n, p, scale, seed, rng_stream);
  return check_launch("kdfm_dropout_bf16");
}

int kdfm_rowscale(const float* x, float* out, int64_t rows, int64_t cols, const float* s, int64_t rows_per_s,
                  float alpha, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && out && s && rows_per_s > 0, "bad args");
  KDFM_1D(rowscale_kernel, rows * cols, x, out, rows, cols, s, rows_per_s, alpha);
  return check_launch("kdfm_rowscale");
}

int kdfm_relu_mask(const float* dy, const float* y, float* out, int64_t n, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && y && out, "null pointer");
  KDFM_1D(relu_mask_kernel, n, dy, y, out, n);
  return check_launch("kdfm_relu_mask");
}

int kdfm_mse(const float* a, const float* b, float* grad, float* loss_acc, int64_t n, float scale, float gscale,
             void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(a && b && loss_acc, "null pointer");
  KDFM_1D(mse_kernel, n, a, b, grad, loss_acc, n, scale, gscale);
  return check_launch("kdfm_mse");
}

int kdfm_l1(const float* a, const float* b, float* grad, float* loss_acc, int64_t n, float scale, float gscale,
            void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(a && b && loss_acc, "null pointer");
  KDFM_1D(l1_kernel, n, a, b, grad, loss_acc, n, scale, gscale);
  return check_launch("kdfm_l1");
}

int kdfm_qkv_prep(const float* qkv, const float* pos_bias_u, const float* pos_bias_v, float* qu, float* qv,
                  int64_t rows, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(qkv && pos_bias_u && pos_bias_v && qu && qv, "null pointer");
  if (d % 4 == 0 && rows * (d / 4) < (int64_t)1 << 31 &&
      ((((uintptr_t)qkv) | ((uintptr_t)pos_bias_u) | ((uintptr_t)pos_bias_v) | ((uintptr_t)qu) | ((uintptr_t)qv)) &
       15) == 0) {
    const int64_t n4 = rows * (d / 4);
    hipLaunchKernelGGL(qkv_prep4_kernel, dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), qkv,
                       pos_bias_u, pos_bias_v, qu, qv, (int)n4, (int)(d / 4));
    return check_launch("kdfm_qkv_prep");
  }
  KDFM_1D(qkv_prep_kernel, rows * d, qkv, pos_bias_u, pos_bias_v, qu, qv, rows, d);
  return check_launch("kdfm_qkv_prep");
}

int kdfm_convw_prep(const float* W, float* fwd, float* bwd, int64_t O, int64_t I, int64_t K, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(W && (fwd || bwd), "null pointer");
  KDFM_1D(convw_prep_kernel, O * I * K, W, fwd, bwd, O, I, K);
  return check_launch("kdfm_convw_prep");
}

int kdfm_convw_grad(const float* G, float* dW, int64_t O, int64_t I, int64_t K, float alpha, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(G && dW, "null pointer");
  KDFM_1D(convw_grad_kernel, O * I * K, G, dW, O, I, K, alpha);
  return check_launch("kdfm_convw_grad");
}

int kdfm_adapter_fwd(const float* zs, const float* h, const float* w2, const float* b2, const float* eps_in, float* zn,
                     float* gamma, int64_t rows, int64_t L, const uint64_t* seed, uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(zs && h && w2 && b2 && zn && gamma, "null pointer");
  KDFM_REQUIRE(eps_in || seed, "need injected eps or a seed");
  KDFM_REQUIRE(L > 0 && L <= 128, "latent dim in (0,128]");
  if (rows == 0) return KDFM_OK;
  hipStream_t st = as_stream(stream);
  if (L % 16 == 0) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(rows, 16), 4096);
    switch (L / 16) {
#define AF_CASE(n)                                                                                                  \
  case n:                                                                                                           \
    hipLaunchKernelGGL(adapter_fwd16_kernel<n>, dim3(grid), dim3(256), 0, st, zs, h, w2, b2, eps_in, zn, gamma, rows, \
                       (int)L, seed, rng_stream);                                                                   \
    break;
      AF_CASE(1) AF_CASE(2) AF_CASE(3) AF_CASE(4) AF_CASE(5) AF_CASE(6) AF_CASE(7) AF_CASE(8)
#undef AF_CASE
    }
    return check_launch("kdfm_adapter_fwd");
  }
  hipLaunchKernelGGL(adapter_fwd_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, st, zs, h, w2,
                     b2, eps_in, zn, gamma, rows, (int)L, seed, rng_stream);
  return check_launch("kdfm_adapter_fwd");
}

int64_t kdfm_adapter_bwd_ws(int64_t rows, int64_t L) {
  const int64_t nb = rows < 16 ? 1 : (kdfm::ceil_div(rows, 16) < kdfm::AB_BLOCKS ? kdfm::ceil_div(rows, 16) : kdfm::AB_BLOCKS);
  return nb * (L + 1);
}

int kdfm_adapter_bwd(const float* dzn, const float* zs, const float* h, const float* gamma, const float* w2,
                     const float* eps_in, float* dzs, float* dh, float* dw2, float* db2, float* ws, int64_t ws_len,
                     int64_t rows, int64_t L, const uint64_t* seed, uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dzn && zs && h && gamma && w2 && dzs && dh && dw2 && db2 && ws, "null pointer");
  KDFM_REQUIRE(eps_in || seed, "need injected eps or a seed");
  KDFM_REQUIRE(L > 0 && L <= 128 && L % 16 == 0, "latent dim a multiple of 16 in (0,128]");
  if (rows == 0) return KDFM_OK;
  int64_t nb = kdfm_adapter_bwd_ws(rows, L) / (L + 1);
  KDFM_REQUIRE(ws_len >= nb * (L + 1), "workspace too small (kdfm_adapter_bwd_ws)");
  const int64_t rp = ceil_div(rows, nb);
  nb = ceil_div(rows, rp);
  hipStream_t st = as_stream(stream);
  switch (L / 16) {
#define AB_CASE(n)                                                                                                  \
  case n:                                                                                                           \
    hipLaunchKernelGGL(adapter_bwd_kernel<n>, dim3((unsigned)nb), dim3(256), 0, st, dzn, zs, h, gamma, w2, eps_in,    \
                       dzs, dh, ws, rows, (int)L, seed, rng_stream, rp);                                             \
    break;
    AB_CASE(1) AB_CASE(2) AB_CASE(3) AB_CASE(4) AB_CASE(5) AB_CASE(6) AB_CASE(7) AB_CASE(8)
#undef AB_CASE
  }
  int rc = check_launch("kdfm_adapter_bwd");
  if (rc) return rc;
  hipLaunchKernelGGL(adapter_bwd_fold_kernel, dim3((unsigned)(L + 1)), dim3(256), 0, st, ws, nb, (int)L, dw2, db2);
  return check_launch("kdfm_adapter_bwd(fold)");
}

int kdfm_fm_step_bias(const float* w_te, const float* b_te, const float* W1, const float* b1, float* cvec, float* evec,
                      int64_t L, int64_t E, int64_t steps, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(w_te && b_te && W1 && b1 && cvec && evec, "null pointer");
  KDFM_REQUIRE(steps >= 1 && steps <= 4096, "steps");
  hipLaunchKernelGGL(fm_step_bias_kernel, dim3((unsigned)steps), dim3(256), 0, as_stream(stream), w_te, b_te, W1, b1,
                     cvec, evec, (int)L, (int)E, (int)steps);
  return check_launch("kdfm_fm_step_bias");
}

int kdfm_fm_time_bwd(const float* dc, const float* evec, const float* W1, float* dW1, float* db1, float* dw_te,
                     float* db_te, int64_t L, int64_t E, int64_t steps, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dc && evec && W1 && dW1 && db1 && dw_te && db_te, "null pointer");
  KDFM_REQUIRE(L >= 1 && L <= 256 && E >= 1 && steps >= 1, "fm_time_bwd: 1 <= L <= 256");
  hipLaunchKernelGGL(fm_time_bwd_kernel, dim3((unsigned)(E + 1)), dim3(256), 0, as_stream(stream), dc, evec, W1, dW1, db1, dw_te, db_te,
                     (int)L, (int)E, (int)steps);
  return check_launch("kdfm_fm_time_bwd");
}

int kdfm_relpos_table(float* pe, int64_t T, int64_t d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(pe && T > 0 && d > 0 && (d % 2) == 0, "bad args");
  KDFM_1D(relpos_table_kernel, (2 * T - 1) * d, pe, T, d);
  return check_launch("kdfm_relpos_table");
}

int kdfm_subsample_lengths(const int64_t* wav_len, int64_t* mel_len, int64_t* len1, int64_t* len2, int64_t B,
                           int64_t hop, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(wav_len && mel_len && hop > 0, "bad args");
  if (B == 0) return KDFM_OK;
  hipLaunchKernelGGL(lengths_kernel, dim3((unsigned)ceil_div(B, 64)), dim3(64), 0, as_stream(stream), wav_len, mel_len,
                     len1, len2, B, hop);
  return check_launch("kdfm_subsample_lengths");
}

int kdfm_step_advance(int64_t* step, uint64_t* seed, void* stream) {
  using namespace kdfm;
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, as_stream(stream), step, seed);
  return check_launch("kdfm_step_advance");
}

}  // extern "C"
