// Strided 1-D unfold / fold (overlap-add) over channels-last rows, for the U-Net FM meta-encoder's
// Conv1d(k 4, stride 2, pad 1) downs and ConvTranspose1d(k 4, stride 2, pad 1) ups (asr_train.py:880-917,
// kdfm/fmmeta.py): a strided conv is unfold + GEMM, its data gradient GEMM + fold; a transposed conv is GEMM +
// fold, its data gradient unfold + GEMM.  Utterances are independent (B blocks of rows); out-of-range taps read
// zero.  Both are HBM-bound elementwise passes (4 B read + 4 B written per element); fold gathers its taps, so
// every output element is written once by one thread (deterministic, no atomics).
#include "common.h"

namespace kdfm {
namespace {

// cols[(b, i)][k * C + c] = x[(b, S i - P + k)][c]  (0 outside [0, Lvalid)); utterance b's rows start at b Lin;
// 4 channels per thread
__global__ __launch_bounds__(256) void unfold1d_kernel(const float* __restrict__ x, int64_t ldx, float* __restrict__ cols,
                                                       int64_t B, int64_t Lin, int64_t Lvalid, int64_t Lrows, int64_t C,
                                                       int K, int S, int P) {
  const int64_t c4n = C / 4;
  const int64_t per_row = (int64_t)K * c4n;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * Lrows * per_row) return;
  const int64_t row = idx / per_row, rem = idx - row * per_row;
  const int k = (int)(rem / c4n);
  const int64_t c = (rem - (int64_t)k * c4n) * 4;
  const int64_t b = row / Lrows, i = row - b * Lrows;
  const int64_t t = S * i - P + k;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t >= 0 && t < Lvalid) v = *reinterpret_cast<const float4*>(x + (b * Lin + t) * ldx + c);
  *reinterpret_cast<float4*>(cols + row * K * C + (int64_t)k * C + c) = v;
}

// out[(b, t)][c] = (R ? R[(b, t)][c] : 0) + [t < Lvalid] (bias ? bias[c] : 0)
//                  + [t < Lvalid] sum_{k : (t + P - k) % S == 0, 0 <= i = (t + P - k) / S < Lrows} cols[(b, i)][k * C + c]
// (Lvalid: the transposed conv's own output length; rows past it are the up path's zero pad, and a tap that
// would land there is cropped by the conv's padding, not added)
__global__ __launch_bounds__(256) void fold1d_kernel(const float* __restrict__ cols, float* __restrict__ out, int64_t ldo,
                                                     const float* __restrict__ bias, const float* __restrict__ R,
                                                     int64_t ldr, int64_t B, int64_t Lrows, int64_t Lout, int64_t Lvalid,
                                                     int64_t C, int K, int S, int P) {
  const int64_t c4n = C / 4;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * Lout * c4n) return;
  const int64_t row = idx / c4n;
  const int64_t c = (idx - row * c4n) * 4;
  const int64_t b = row / Lout, t = row - b * Lout;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (R) acc = *reinterpret_cast<const float4*>(R + row * ldr + c);
  if (t < Lvalid) {
    if (bias) {
      const float4 bb = *reinterpret_cast<const float4*>(bias + c);
      acc.x += bb.x; acc.y += bb.y; acc.z += bb.z; acc.w += bb.w;
    }
    for (int k = 0; k < K; ++k) {   // taps in order: a fixed summation order
      const int64_t u = t + P - k;
      if (u < 0 || u % S) continue;
      const int64_t i = u / S;
      if (i >= Lrows) continue;
      const float4 v = *reinterpret_cast<const float4*>(cols + (b * Lrows + i) * K * C + (int64_t)k * C + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  *reinterpret_cast<float4*>(out + row * ldo + c) = acc;
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_unfold1d(const float* x, int64_t ldx, float* cols, int64_t B, int64_t Lin, int64_t Lvalid, int64_t Lrows,
                  int64_t C, int32_t K, int32_t S, int32_t P, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && cols, "null pointer");
  KDFM_REQUIRE(C > 0 && C % 4 == 0 && ldx >= C && ldx % 4 == 0, "C and ldx must be multiples of 4 (ldx >= C)");
  KDFM_REQUIRE(K > 0 && K <= 16 && S > 0 && P >= 0, "bad taps / stride / pad");
  KDFM_REQUIRE(Lvalid >= 0 && Lvalid <= Lin, "Lvalid must be in [0, Lin]");
  KDFM_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)cols & 15) == 0, "operands must be 16-byte aligned");
  const int64_t n = B * Lrows * K * (C / 4);
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(unfold1d_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), x, ldx, cols, B,
                     Lin, Lvalid, Lrows, C, (int)K, (int)S, (int)P);
  return check_launch("kdfm_unfold1d");
}

int kdfm_fold1d(const float* cols, float* out, int64_t ldo, const float* bias, const float* R, int64_t ldr, int64_t B,
                int64_t Lrows, int64_t Lout, int64_t Lvalid, int64_t C, int32_t K, int32_t S, int32_t P, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(cols && out, "null pointer");
  KDFM_REQUIRE(C > 0 && C % 4 == 0 && ldo >= C && ldo % 4 == 0 && (!R || (ldr >= C && ldr % 4 == 0)),
               "C, ldo, ldr must be multiples of 4");
  KDFM_REQUIRE(K > 0 && K <= 16 && S > 0 && P >= 0, "bad taps / stride / pad");
  KDFM_REQUIRE((((uintptr_t)cols | (uintptr_t)out | (uintptr_t)bias | (uintptr_t)R) & 15) == 0,
               "operands must be 16-byte aligned");
  const int64_t n = B * Lout * (C / 4);
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(fold1d_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), cols, out, ldo,
                     bias, R, ldr, B, Lrows, Lout, Lvalid, C, (int)K, (int)S, (int)P);
  return check_launch("kdfm_fold1d");
}

}  // extern "C"
