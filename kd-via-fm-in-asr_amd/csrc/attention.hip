// Relative-position attention score normalisation (NeMo RelPositionMultiHeadAttention,
// Appendix A.7; rel_shift and forward_attention semantics).  The two score matrices come from
// MFMA GEMMs: AC = (q+u)K^T (B,H,T,T) and BD = (q+v)P^T (B,H,T,2T-1).  rel_shift is folded into
// the index math: bd_shift[i][j] = BD[i][T-1-i+j].  Masked scores are -1e4 before the softmax and
// the probabilities are re-zeroed (fully padded query rows -> all zero), then inverted dropout
// (dropout_att) with a counter-RNG mask that the backward regenerates.
#include "common.h"

namespace kdfm {
namespace {

constexpr int MAXE = 8;  // T <= 512 per row (64 lanes x 8)

__global__ __launch_bounds__(256) void relpos_softmax_fwd_kernel(
    const float* __restrict__ ac, const float* __restrict__ bd, const int64_t* __restrict__ lens,
    float* __restrict__ P, float* __restrict__ Pd, int64_t B, int64_t H, int T, float scale, float p_drop,
    const uint64_t* seed_ptr, uint64_t rng_stream) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // (b*H + h)*T + i
  if (row >= B * H * T) return;
  const int i = (int)(row % T);
  const int64_t bh = row / T;
  const int64_t b = bh / H;
  const int64_t len = lens ? lens[b] : T;
  const float* acr = ac + row * T;
  const float* bdr = bd + row * (int64_t)(2 * T - 1);
  float* pr = P + row * T;
  float* pdr = Pd ? Pd + row * T : nullptr;
  if (i >= len) {
    for (int j = lane; j < T; j += 64) {
      pr[j] = 0.f;
      if (pdr) pdr[j] = 0.f;
    }
    return;
  }
  float s[MAXE];
  float mx = -3.0e38f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + 64 * e;
    if (j < T && j < len) {
      s[e] = (acr[j] + bdr[T - 1 - i + j]) * scale;
      mx = fmaxf(mx, s[e]);
    } else {
      s[e] = -3.0e38f;
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + 64 * e;
    s[e] = (j < T && j < len) ? __expf(s[e] - mx) : 0.f;
    sum += s[e];
  }
  const float inv = 1.f / wave_sum(sum);
  uint64_t seed = 0;
  float keep_scale = 1.f;
  if (pdr && p_drop > 0.f) {
    seed = load_seed(seed_ptr);
    keep_scale = 1.f / (1.f - p_drop);
  }
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + 64 * e;
    if (j < T) {
      const float pv = s[e] * inv;
      pr[j] = pv;
      if (pdr) {
        pdr[j] = (p_drop > 0.f && !attn_drop_keep(rng_key(seed, rng_stream), attn_drop_rowpairs(row, T), j, p_drop))
                     ? 0.f : pv * keep_scale;
      }
    }
  }
}

// dS = P*(dP - sum_j P dP) * scale ; dAC = dS ; dBD[i][T-1-i+j] = dS[i][j], zero elsewhere
__global__ __launch_bounds__(256) void relpos_softmax_bwd_kernel(
    const float* __restrict__ P, const float* __restrict__ dPd, float* __restrict__ dAC, float* __restrict__ dBD,
    int64_t rows, int T, float scale, float p_drop, const uint64_t* seed_ptr, uint64_t rng_stream) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int i = (int)(row % T);
  const float* pr = P + row * T;
  const float* dr = dPd + row * T;
  uint64_t seed = 0;
  float keep_scale = 1.f;
  if (p_drop > 0.f) {
    seed = load_seed(seed_ptr);
    keep_scale = 1.f / (1.f - p_drop);
  }
  float pv[MAXE], dv[MAXE];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + 64 * e;
    if (j < T) {
      pv[e] = pr[j];
      float g = dr[j];
      if (p_drop > 0.f) {
        g = attn_drop_keep(rng_key(seed, rng_stream), attn_drop_rowpairs(row, T), j, p_drop) ? g * keep_scale : 0.f;
      }
      dv[e] = g;
      dot += pv[e] * g;
    } else {
      pv[e] = 0.f;
      dv[e] = 0.f;
    }
  }
  dot = wave_sum(dot);
  float* dacr = dAC + row * T;
  float* dbdr = dBD + row * (int64_t)(2 * T - 1);
  const int off = T - 1 - i;
  // zero the parts of the dBD row that no key touches: [0, off) and [off+T, 2T-1)
  for (int q = lane; q < off; q += 64) dbdr[q] = 0.f;
  for (int q = off + T + lane; q < 2 * T - 1; q += 64) dbdr[q] = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = lane + 64 * e;
    if (j < T) {
      const float ds = pv[e] * (dv[e] - dot) * scale;
      dacr[j] = ds;
      dbdr[off + j] = ds;
    }
  }
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_relpos_softmax_fwd(const float* ac, const float* bd, const int64_t* lengths, float* P, float* Pdrop,
                            int64_t B, int64_t H, int64_t T, float scale, float dropout_p, const uint64_t* seed,
                            uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(ac && bd && P, "null pointer");
  KDFM_REQUIRE(T > 0 && T <= 64 * MAXE, "T must be in (0, 512]");
  KDFM_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "dropout p");
  const int64_t rows = B * H * T;
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(relpos_softmax_fwd_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream),
                     ac, bd, lengths, P, Pdrop, B, H, (int)T, scale, dropout_p, seed, rng_stream);
  return check_launch("kdfm_relpos_softmax_fwd");
}

int kdfm_relpos_softmax_bwd(const float* P, const float* dPdrop, float* dAC, float* dBD, int64_t B, int64_t H,
                            int64_t T, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                            void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(P && dPdrop && dAC && dBD, "null pointer");
  KDFM_REQUIRE(T > 0 && T <= 64 * MAXE, "T must be in (0, 512]");
  const int64_t rows = B * H * T;
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(relpos_softmax_bwd_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream),
                     P, dPdrop, dAC, dBD, rows, (int)T, scale, dropout_p, seed, rng_stream);
  return check_launch("kdfm_relpos_softmax_bwd");
}

}  // extern "C"
