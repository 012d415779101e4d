// Depthwise-separable ('dw_striding') convolution subsampling: the stride-2 3x3 convolutions of
// NeMo ConvSubsampling(subsampling='dw_striding') (built at conformer_encoder.py:381-390, recipe
// fast-conformer_ctc_bpe.yaml:122-125; module source absent, restated in oracle/ver5.py
// subsampling_dw_striding) on channels-last activations (B, T, F, C):
//   stage 0: Conv2d(1 -> C, 3x3, s2)          -> ReLU     (Cin = 1: the input channel broadcast)
//   stage s: depthwise Conv2d(C, 3x3, s2, g=C) -> pointwise 1x1 (kdfm_gemm) -> ReLU
// with NeMo's masked conv sequence: frames at or past a layer's valid length are zero before the
// layer reads them and after it writes them.  The pointwise 1x1 convs and the output Linear are
// plain GEMMs (kdfm_gemm, EPI_ROWMASK), so only the 3x3 stride-2 layers live here.
//
// These layers are HBM-bound (9 MACs per element read): one thread per 4 channels of one output
// position, float4 loads along the channel axis (coalesced across the wave), the 3x3 window's
// re-reads served by L1/L2.  The weight gradient is an ordered two-pass reduction (per-slab
// partials, then a fixed-order fold) — deterministic in every mode.
#include "common.h"

namespace kdfm {
namespace {

constexpr int DW_NT = 256;
constexpr int DW_K = 10;  // 9 taps + bias

__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
  return a >= 0 ? a / b : -((-a + b - 1) / b);
}

__global__ void conv_lengths_kernel(const int64_t* __restrict__ in, int64_t* __restrict__ out, int64_t n,
                                    int pad_total, int kernel, int stride) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = floor_div(in[i] + pad_total - kernel, stride) + 1;
}

// y[b, to, fo, c..c+3] = act(bias + sum_{i,j} w[c, i, j] * x[b, 2 to - pt + i, 2 fo - pf + j, c or 0])
// A thread owns 4 channels of DWS_P consecutive output columns fo: its 36 taps and 4 biases are loaded once and
// reused DWS_P times (one thread per output float4 re-read them from cache for every position: 45 loads per 4
// outputs, 3.35 ms per FastConformer-XL first-stage launch, profiles/r06/r6e); lanes run over the channel groups,
// so a wave's stores are contiguous and the broadcast input (BCAST) is one address per wave.
constexpr int DWS_P = 8;
template <bool BCAST>
__global__ __launch_bounds__(DW_NT) void dws_fwd_kernel(const float* __restrict__ x, const int64_t* __restrict__ in_len,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        float* __restrict__ y, const int64_t* __restrict__ out_len,
                                                        int64_t B, int Ti, int Fi, int C, int To, int Fo, int pt, int pf,
                                                        int relu) {
  const int CV = C >> 2;
  const int FB = (Fo + DWS_P - 1) / DWS_P;
  int64_t idx = (int64_t)blockIdx.x * DW_NT + threadIdx.x;
  if (idx >= B * To * FB * CV) return;
  const int cg = (int)(idx % CV);
  int64_t r = idx / CV;
  const int fb = (int)(r % FB);
  r /= FB;
  const int to = (int)(r % To);
  const int64_t b = r / To;
  const int c = cg * 4;
  const bool live = !out_len || to < out_len[b];
  float wv[4][9];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 9; ++k) wv[q][k] = w[(c + q) * 9 + k];
  const float4 bs = *reinterpret_cast<const float4*>(bias + c);
  const int64_t lin = in_len ? in_len[b] : Ti;
#pragma unroll
  for (int pp = 0; pp < DWS_P; ++pp) {
    const int fo = fb * DWS_P + pp;
    if (fo >= Fo) break;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
      acc = bs;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int ti = 2 * to - pt + i;
        if (ti < 0 || ti >= Ti || ti >= lin) continue;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int fi = 2 * fo - pf + j;
          if (fi < 0 || fi >= Fi) continue;
          const int64_t pos = (b * Ti + ti) * Fi + fi;
          float4 xv;
          if constexpr (BCAST) {
            const float s = x[pos];
            xv = make_float4(s, s, s, s);
          } else {
            xv = *reinterpret_cast<const float4*>(x + pos * C + c);
          }
          const int k = i * 3 + j;
          acc.x += wv[0][k] * xv.x;
          acc.y += wv[1][k] * xv.y;
          acc.z += wv[2][k] * xv.z;
          acc.w += wv[3][k] * xv.w;
        }
      }
      if (relu) {
        acc.x = fmaxf(acc.x, 0.f);
        acc.y = fmaxf(acc.y, 0.f);
        acc.z = fmaxf(acc.z, 0.f);
        acc.w = fmaxf(acc.w, 0.f);
      }
    }
    *reinterpret_cast<float4*>(y + (((b * To + to) * Fo + fo) * (int64_t)C + c)) = acc;
  }
}

// dx[b, ti, fi, c] = relu'(xs) * sum over the (<= 2x2) outputs whose window covers (ti, fi) of
// dy[b, to, fo, c] * w[c, ti + pt - 2 to, fi + pf - 2 fo]; zero at ti >= in_len (masked input).
__global__ __launch_bounds__(DW_NT) void dws_dgrad_kernel(const float* __restrict__ dy, const int64_t* __restrict__ out_len,
                                                          const float* __restrict__ w, const float* __restrict__ xs,
                                                          const int64_t* __restrict__ in_len, float* __restrict__ dx,
                                                          int64_t B, int Ti, int Fi, int C, int To, int Fo, int pt,
                                                          int pf) {
  const int CV = C >> 2;
  int64_t idx = (int64_t)blockIdx.x * DW_NT + threadIdx.x;
  if (idx >= B * Ti * Fi * CV) return;
  const int cg = (int)(idx % CV);
  int64_t r = idx / CV;
  const int fi = (int)(r % Fi);
  r /= Fi;
  const int ti = (int)(r % Ti);
  const int64_t b = r / Ti;
  const int c = cg * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!in_len || ti < in_len[b]) {
    const int64_t lout = out_len ? out_len[b] : To;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int t2 = ti + pt - i;
      if (t2 < 0 || (t2 & 1)) continue;
      const int to = t2 >> 1;
      if (to >= To || to >= lout) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int f2 = fi + pf - j;
        if (f2 < 0 || (f2 & 1)) continue;
        const int fo = f2 >> 1;
        if (fo >= Fo) continue;
        const float4 g = *reinterpret_cast<const float4*>(dy + ((b * To + to) * Fo + fo) * C + c);
        const int k = i * 3 + j;
        acc.x += w[(c + 0) * 9 + k] * g.x;
        acc.y += w[(c + 1) * 9 + k] * g.y;
        acc.z += w[(c + 2) * 9 + k] * g.z;
        acc.w += w[(c + 3) * 9 + k] * g.w;
      }
    }
    if (xs) {
      const float4 s = *reinterpret_cast<const float4*>(xs + idx * 4);
      acc.x = s.x > 0.f ? acc.x : 0.f;
      acc.y = s.y > 0.f ? acc.y : 0.f;
      acc.z = s.z > 0.f ? acc.z : 0.f;
      acc.w = s.w > 0.f ? acc.w : 0.f;
    }
  }
  *reinterpret_cast<float4*>(dx + idx * 4) = acc;
}

// Weight-gradient partials: block s reduces output rows [s*slab, (s+1)*slab) of (b, to, fo) into
// part[s][k][c], k = 9 taps + bias.  Threads = CT channel groups (4 channels each) x RG row groups;
// the row groups are combined in LDS in a fixed order.
template <bool BCAST>
__global__ __launch_bounds__(DW_NT) void dws_wgrad_part_kernel(const float* __restrict__ dy, const int64_t* __restrict__ out_len,
                                                               const float* __restrict__ x, const int64_t* __restrict__ in_len,
                                                               float* __restrict__ part, int64_t B, int Ti, int Fi, int C,
                                                               int To, int Fo, int pt, int pf, int64_t slab) {
  extern __shared__ float red[];  // [RG][CT][DW_K*4]
  const int CT = C >> 2;
  const int RG = DW_NT / CT;
  const int tid = threadIdx.x;
  const int cg = tid % CT;
  const int rg = tid / CT;
  const int c = cg * 4;
  float acc[DW_K][4];
#pragma unroll
  for (int k = 0; k < DW_K; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[k][v] = 0.f;
  const int64_t rows = B * To * Fo;
  const int64_t r0 = (int64_t)blockIdx.x * slab;
  const int64_t r1 = r0 + slab < rows ? r0 + slab : rows;
  if (rg < RG) {
    for (int64_t r = r0 + rg; r < r1; r += RG) {
      const int fo = (int)(r % Fo);
      const int64_t bt = r / Fo;
      const int to = (int)(bt % To);
      const int64_t b = bt / To;
      if (out_len && to >= out_len[b]) continue;
      const float4 g = *reinterpret_cast<const float4*>(dy + r * C + c);
      acc[9][0] += g.x;
      acc[9][1] += g.y;
      acc[9][2] += g.z;
      acc[9][3] += g.w;
      const int64_t lin = in_len ? in_len[b] : Ti;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int ti = 2 * to - pt + i;
        if (ti < 0 || ti >= Ti || ti >= lin) continue;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int fi = 2 * fo - pf + j;
          if (fi < 0 || fi >= Fi) continue;
          const int64_t pos = (b * Ti + ti) * Fi + fi;
          float4 xv;
          if constexpr (BCAST) {
            const float s = x[pos];
            xv = make_float4(s, s, s, s);
          } else {
            xv = *reinterpret_cast<const float4*>(x + pos * C + c);
          }
          const int k = i * 3 + j;
          acc[k][0] += g.x * xv.x;
          acc[k][1] += g.y * xv.y;
          acc[k][2] += g.z * xv.z;
          acc[k][3] += g.w * xv.w;
        }
      }
    }
    float* mine = red + ((int64_t)rg * CT + cg) * (DW_K * 4);
#pragma unroll
    for (int k = 0; k < DW_K; ++k)
#pragma unroll
      for (int v = 0; v < 4; ++v) mine[k * 4 + v] = acc[k][v];
  }
  __syncthreads();
  // fixed-order combine over the row groups: thread t < CT*DW_K*4 owns one (c, k, v) value
  for (int e = tid; e < CT * DW_K * 4; e += DW_NT) {
    const int g = e / (DW_K * 4);
    const int kv = e % (DW_K * 4);
    float s = 0.f;
    for (int q = 0; q < RG; ++q) s += red[((int64_t)q * CT + g) * (DW_K * 4) + kv];
    const int k = kv >> 2, v = kv & 3;
    part[((int64_t)blockIdx.x * DW_K + k) * C + g * 4 + v] = s;
  }
}

// dw[c*9 + k] (+)= sum_s part[s][k][c]; db[c] (+)= sum_s part[s][9][c], slabs in order.
__global__ __launch_bounds__(DW_NT) void dws_wgrad_fold_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                               float* __restrict__ db, int C, int64_t S, int accumulate) {
  const int e = blockIdx.x * DW_NT + threadIdx.x;
  if (e >= C * DW_K) return;
  const int k = e / C, c = e % C;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int64_t s = 0;
  // four independent chains over interleaved slabs, combined in a fixed order
  for (; s + 4 <= S; s += 4) {
    s0 += part[((s + 0) * DW_K + k) * C + c];
    s1 += part[((s + 1) * DW_K + k) * C + c];
    s2 += part[((s + 2) * DW_K + k) * C + c];
    s3 += part[((s + 3) * DW_K + k) * C + c];
  }
  for (; s < S; ++s) s0 += part[(s * DW_K + k) * C + c];
  const float tot = (s0 + s1) + (s2 + s3);
  float* dst = k < 9 ? dw + (int64_t)c * 9 + k : db + c;
  *dst = accumulate ? *dst + tot : tot;
}

int64_t wgrad_slabs(int64_t rows) {
  int64_t s = ceil_div(rows, 256);
  return s < 1024 ? (s < 1 ? 1 : s) : 1024;
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_conv_lengths(const int64_t* in, int64_t* out, int64_t n, int32_t pad_total, int32_t kernel, int32_t stride,
                      void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(in && out && n >= 0 && kernel > 0 && stride > 0, "bad args");
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(conv_lengths_kernel, dim3((unsigned)ceil_div(n, 64)), dim3(64), 0, as_stream(stream), in, out, n,
                     pad_total, kernel, stride);
  return check_launch("kdfm_conv_lengths");
}

static int dws_check(int64_t B, int64_t Ti, int64_t Fi, int64_t Cin, int64_t C, int64_t To, int64_t Fo, int32_t pt,
                     int32_t pf) {
  using namespace kdfm;
  KDFM_REQUIRE(B >= 0 && Ti > 0 && Fi > 0 && To > 0 && Fo > 0, "bad sizes");
  KDFM_REQUIRE(C > 0 && C % 4 == 0 && C <= 1024, "channels must be a positive multiple of 4 (<= 1024)");
  KDFM_REQUIRE(Cin == 1 || Cin == C, "input channels must be 1 (first stage) or C (depthwise)");
  KDFM_REQUIRE(pt >= 0 && pt <= 2 && pf >= 0 && pf <= 2, "padding must be in [0, 2]");
  // every output window must start inside the padded input (the conv output size formula)
  KDFM_REQUIRE(2 * (To - 1) - pt < Ti && 2 * (Fo - 1) - pf < Fi, "output larger than the input allows");
  KDFM_REQUIRE(Ti < (1 << 30) && Fi < (1 << 30), "sizes too large");
  return KDFM_OK;
}

int kdfm_dwsub_conv(const float* x, const int64_t* in_len, const float* w, const float* bias, float* y,
                    const int64_t* out_len, int64_t B, int64_t Ti, int64_t Fi, int64_t Cin, int64_t C, int64_t To,
                    int64_t Fo, int32_t pad_t, int32_t pad_f, int32_t relu, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && w && bias && y, "null pointer");
  KDFM_REQUIRE(((uintptr_t)bias | (uintptr_t)y | (Cin == 1 ? 0 : (uintptr_t)x)) % 16 == 0, "operands must be 16-byte aligned");
  int rc = dws_check(B, Ti, Fi, Cin, C, To, Fo, pad_t, pad_f);
  if (rc) return rc;
  const int64_t n = B * To * ceil_div(Fo, DWS_P) * (C / 4);
  if (n == 0) return KDFM_OK;
  dim3 grid((unsigned)ceil_div(n, DW_NT));
  if (Cin == 1)
    hipLaunchKernelGGL(dws_fwd_kernel<true>, grid, dim3(DW_NT), 0, as_stream(stream), x, in_len, w, bias, y, out_len, B,
                       (int)Ti, (int)Fi, (int)C, (int)To, (int)Fo, pad_t, pad_f, relu);
  else
    hipLaunchKernelGGL(dws_fwd_kernel<false>, grid, dim3(DW_NT), 0, as_stream(stream), x, in_len, w, bias, y, out_len,
                       B, (int)Ti, (int)Fi, (int)C, (int)To, (int)Fo, pad_t, pad_f, relu);
  return check_launch("kdfm_dwsub_conv");
}

int kdfm_dwsub_conv_dgrad(const float* dy, const int64_t* out_len, const float* w, const float* x_saved,
                          const int64_t* in_len, float* dx, int64_t B, int64_t Ti, int64_t Fi, int64_t C, int64_t To,
                          int64_t Fo, int32_t pad_t, int32_t pad_f, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && w && dx, "null pointer");
  KDFM_REQUIRE(((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)x_saved) % 16 == 0, "operands must be 16-byte aligned");
  int rc = dws_check(B, Ti, Fi, C, C, To, Fo, pad_t, pad_f);
  if (rc) return rc;
  const int64_t n = B * Ti * Fi * (C / 4);
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(dws_dgrad_kernel, dim3((unsigned)ceil_div(n, DW_NT)), dim3(DW_NT), 0, as_stream(stream), dy,
                     out_len, w, x_saved, in_len, dx, B, (int)Ti, (int)Fi, (int)C, (int)To, (int)Fo, pad_t, pad_f);
  return check_launch("kdfm_dwsub_conv_dgrad");
}

int64_t kdfm_dwsub_conv_wgrad_ws(int64_t B, int64_t To, int64_t Fo, int64_t C) {
  return kdfm::wgrad_slabs(B * To * Fo) * kdfm::DW_K * C;
}

int kdfm_dwsub_conv_wgrad(const float* dy, const int64_t* out_len, const float* x, const int64_t* in_len, float* dw,
                          float* db, float* ws, int64_t ws_len, int64_t B, int64_t Ti, int64_t Fi, int64_t Cin,
                          int64_t C, int64_t To, int64_t Fo, int32_t pad_t, int32_t pad_f, int32_t accumulate,
                          void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && x && dw && db && ws, "null pointer");
  KDFM_REQUIRE(((uintptr_t)dy | (Cin == 1 ? 0 : (uintptr_t)x)) % 16 == 0, "operands must be 16-byte aligned");
  int rc = dws_check(B, Ti, Fi, Cin, C, To, Fo, pad_t, pad_f);
  if (rc) return rc;
  KDFM_REQUIRE(C / 4 <= DW_NT, "too many channels for one block");
  const int64_t rows = B * To * Fo;
  const int64_t S = wgrad_slabs(rows);
  KDFM_REQUIRE(ws_len >= S * DW_K * C, "workspace too small (kdfm_dwsub_conv_wgrad_ws)");
  const int64_t slab = ceil_div(rows > 0 ? rows : 1, S);
  const int CT = (int)(C / 4);
  const size_t shmem = (size_t)(DW_NT / CT) * CT * DW_K * 4 * sizeof(float);
  hipStream_t st = as_stream(stream);
  if (Cin == 1)
    hipLaunchKernelGGL(dws_wgrad_part_kernel<true>, dim3((unsigned)S), dim3(DW_NT), shmem, st, dy, out_len, x, in_len,
                       ws, B, (int)Ti, (int)Fi, (int)C, (int)To, (int)Fo, pad_t, pad_f, slab);
  else
    hipLaunchKernelGGL(dws_wgrad_part_kernel<false>, dim3((unsigned)S), dim3(DW_NT), shmem, st, dy, out_len, x, in_len,
                       ws, B, (int)Ti, (int)Fi, (int)C, (int)To, (int)Fo, pad_t, pad_f, slab);
  rc = check_launch("kdfm_dwsub_conv_wgrad");
  if (rc) return rc;
  hipLaunchKernelGGL(dws_wgrad_fold_kernel, dim3((unsigned)ceil_div(C * DW_K, DW_NT)), dim3(DW_NT), 0, st, ws, dw, db,
                     (int)C, S, accumulate);
  return check_launch("kdfm_dwsub_conv_wgrad(fold)");
}

}  // extern "C"
