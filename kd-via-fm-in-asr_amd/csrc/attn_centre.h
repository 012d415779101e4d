// Key / value centring of the fused relative-position attention (attn_fused.hip forward, attn_bwd.hip dQ
// kernel).  K and V enter the bf16 MFMAs as K_j - kc and V_j - vc, kc / vc = the mean of the utterance's
// first n key / value rows (this head's columns), n = min(length, 16) rounded down to a power of two.
// Scores move by q_i . kc, the same along a row, so softmax is unchanged; O_i = sum_j Pd_ij (V_j - vc) +
// (sum_j Pd_ij) vc and dPd_ij = dO_i . (V_j - vc) + dO_i . vc with the second terms in f32.  A component
// the keys / values share (a per-channel offset common to all frames) then never goes through the bf16
// rounding, whose error it would scale (7 % on the FastConformer layer-0 q/k gradients before,
// tools/attn_small_diag.py); a mean rather than one row keeps zero-mean keys' rounding error unchanged.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace kdfm {

// c[0][0..dk) = kc, c[1][0..dk) = vc (zeros for an empty utterance); W >= dk is the centre table's width
// (the kernel's padded head dim).  Every thread of the block must call it (ends with a barrier); rows are
// summed in order by one thread per float4 column group, so the forward and the backward compute the same
// bits.
template <int W>
__device__ __forceinline__ void kv_centre(const float* kbase, const float* vbase, int64_t ld, int len, int dk,
                                          float (*c)[W]) {
  const int cq = dk >> 2;
  const int t = threadIdx.x;
  if (t < 2 * cq) {
    const bool isv = t >= cq;
    const int c4 = (isv ? t - cq : t) * 4;
    const float* src = (isv ? vbase : kbase) + c4;
    const int n = len >= 16 ? 16 : len >= 8 ? 8 : len >= 4 ? 4 : len >= 2 ? 2 : (len > 0 ? 1 : 0);
    // all 16 loads in flight at once (clamped rows, masked by a multiply; adding the zeros of rows >= n
    // leaves the in-order sum unchanged)
    float4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = *reinterpret_cast<const float4*>(src + (int64_t)(r < n ? r : 0) * ld);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float m = r < n ? 1.f : 0.f;
      s.x += m * v[r].x; s.y += m * v[r].y; s.z += m * v[r].z; s.w += m * v[r].w;
    }
    const float inv = n > 0 ? 1.f / (float)n : 0.f;   // a power of two: exact
    float* o = c[isv ? 1 : 0] + c4;
    o[0] = s.x * inv; o[1] = s.y * inv; o[2] = s.z * inv; o[3] = s.w * inv;
  }
  __syncthreads();
}

// Prepared bf16 operands of the attention kernels (csrc/attn_fwd3.hip kdfm_attn_kv_prep / kdfm_attn_band_prep):
// key / value tiles (B*H, attn_prep_tp(T), LR) and band rows (layers*H, attn_prep_npb(T), LR) with
// kAttnBandPad0 zero rows before position 0 and kAttnBandPad1 after the last (the forward stages 128 band
// rows per step, the dQ kernel 144 rounded up to whole 1 KB DMA chunks: up to 149 rows past the step's first)
constexpr int kAttnBandPad0 = 64;
constexpr int kAttnBandPad1 = 88;
__host__ __device__ inline int64_t attn_prep_tp(int64_t T) { return (T + 63) / 64 * 64; }
__host__ __device__ inline int64_t attn_prep_npb(int64_t T) { return kAttnBandPad0 + (2 * T - 1) + kAttnBandPad1; }
// padded head dim of the prepared tiles: 48 (a 32-wide and a 16-wide MFMA k-step) for head dims <= 48 -- the
// bench's student / teacher (44) -- else 64 or 128
__host__ __device__ inline int attn_prep_dkp(int64_t dk) { return dk > 64 ? 128 : dk > 48 ? 64 : 48; }

}  // namespace kdfm
