// Output-side losses of the ver5 step:
//   log_softmax of the ConvASRDecoder logits (conv_asr.py:456-468),
//   CTC (NeMo CTCLoss -> torch CTCLoss, losses/ctc.py:68-82; blank = V, zero_infinity, mean_batch
//   from ctc_models.py:81-85) with its logits gradient exp(lp) - posterior,
//   logit KD (asr_train_diffm.py:751-756: kl_div(log_softmax(s/T), softmax(t/T), 'batchmean') * T^2),
//   and the final loss assembly (asr_train_diffm.py:803-811).
#include <climits>
#include <math.h>

#include <type_traits>

#include "common.h"

namespace kdfm {
namespace {

constexpr float NEG_INF = -INFINITY;

__device__ __forceinline__ float lse2(float a, float b) {
  if (a == NEG_INF) return b;
  if (b == NEG_INF) return a;
  const float m = fmaxf(a, b);
  return m + log1pf(__expf(-fabsf(a - b)));
}

// the CTC recursions' log-add on the hardware exp / log (v_exp_f32, v_log_f32), branch-free: a frame of the
// alpha / beta chain is this function twice per state, so its latency is the recursion's.  log(1 + e) for
// e = exp(-|a - b|) in (0, 1] differs from log1pf(e) by < 1e-7 absolute, below the f32 resolution of the
// running sums (|alpha| ~ 1e2..1e3); an operand of -inf returns the other exactly (e = 0, log(1) = 0)
__device__ __forceinline__ float lse2_fast(float a, float b) {
  const float m = fmaxf(a, b);
  const float e = __expf(fminf(a, b) - m);
  const float r = m + __logf(1.f + e);
  return m == NEG_INF ? NEG_INF : r;
}

// one wave per row, NV = ceil(C / 64) values per lane in registers (vocabularies up to 4096 classes:
// the decoder width V+1 comes from the teacher's tokenizer, conformer_ctc_bpe.yaml:87)
template <int NV>
__global__ __launch_bounds__(256) void log_softmax_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t rows,
                                                          int C, int64_t ldx, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float v[NV];
  float mx = NEG_INF;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < C) ? x[r * ldx + c] : NEG_INF;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (lane + 64 * i < C) ? __expf(v[i] - mx) : 0.f;
  const float lz = mx + __logf(wave_sum(s));
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) y[r * ldy + c] = v[i] - lz;
  }
}

// greedy CTC predictions: idx[r] = argmax_c x[r, c]   (log_probs.argmax(-1), asr_train_diffm.py:635)
__global__ __launch_bounds__(256) void argmax_kernel(const float* __restrict__ x, int64_t* __restrict__ idx,
                                                     int64_t rows, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = x[r * C + c];
    if (v > best) { best = v; bi = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) idx[r] = bi;
}

// dx = dy - exp(y) * sum(dy)   (log_softmax backward, y = log_softmax output)
template <int NV>
__global__ __launch_bounds__(256) void log_softmax_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                              float* __restrict__ dx, int64_t rows, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float g[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    g[i] = (c < C) ? dy[r * C + c] : 0.f;
    s += g[i];
  }
  s = wave_sum(s);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) dx[r * C + c] = g[i] - __expf(y[r * C + c]) * s;
  }
}

// CTC in two launches (the alpha / beta recursions are latency-bound chains over the frames):
//  ctc_ab_kernel, grid (B, 2): y = 0 runs the alpha recursion forwards and y = 1 the beta recursion
//    backwards, concurrently.  SPT states per thread; the emissions of CH frames are gathered into
//    registers per chunk (one memory latency per CH frames instead of one per frame), the chunk's
//    alpha / beta values stay in registers and are stored at the chunk's end, and one barrier per
//    frame orders the ping-pong LDS rows.  The alpha block also writes the utterance's nll.
//  ctc_grad_kernel, grid (B, ceil(T / CTC_FPB)): posteriors and the logits gradient, independent
//    across frames.  Workspaces alpha / beta (B, T, 2 Umax + 1) in log space; nll (B);
//    grad (B, T, C) = scale * (exp(lp) - posterior) for t < len, 0 beyond (all 0 / NaN if infeasible).
// Same recursions, the same log-add order and the same fixed-order posterior sums as a single-block
// formulation: the result is bitwise reproducible.
constexpr int CTC_FPB = 4;

__device__ __forceinline__ int ctc_label(const int64_t* tg, int64_t s, int blank) {
  return (s & 1) ? (int)tg[s >> 1] : blank;
}

template <int SPT, int CH>
__global__ __launch_bounds__(1024) void ctc_ab_kernel(const float* __restrict__ lp, const int64_t* __restrict__ targets,
                                                      const int64_t* __restrict__ in_len,
                                                      const int64_t* __restrict__ tgt_len, float* __restrict__ alpha,
                                                      float* __restrict__ beta, float* __restrict__ nll_out, int64_t T,
                                                      int C, int64_t Umax, int blank, int zero_inf) {
  extern __shared__ float sh[];
  const int64_t b = blockIdx.x;
  const bool bwd = blockIdx.y == 1;
  const int64_t S_max = 2 * Umax + 1;
  const int64_t U = tgt_len[b] < Umax ? tgt_len[b] : Umax;
  const int S = (int)(2 * U + 1);
  const int64_t Tb = in_len[b] < T ? in_len[b] : T;
  if (Tb <= 0) {
    if (!bwd && threadIdx.x == 0) nll_out[b] = (U == 0 || !zero_inf) ? (U == 0 ? 0.f : INFINITY) : 0.f;
    return;
  }
  const float* lpb = lp + b * T * C;
  const int64_t* tg = targets + b * Umax;
  float* out = (bwd ? beta : alpha) + b * T * S_max;
  float* cur = sh;
  float* nxt = sh + S_max;
  int lab[SPT];
  bool skip[SPT];
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int s = threadIdx.x + k * blockDim.x;
    lab[k] = blank;
    skip[k] = false;
    if (s < S) {
      lab[k] = ctc_label(tg, s, blank);
      if (!bwd) skip[k] = s >= 2 && lab[k] != blank && lab[k] != ctc_label(tg, s - 2, blank);
      else skip[k] = s + 2 < S && lab[k] != blank && lab[k] != ctc_label(tg, s + 2, blank);
    }
  }
  const int64_t tfirst = bwd ? Tb - 1 : 0;
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int s = threadIdx.x + k * blockDim.x;
    if (s < S) {
      float v = NEG_INF;
      if (!bwd) {
        if (s == 0) v = lpb[blank];
        if (s == 1) v = lpb[lab[k]];
      } else {
        if (s == S - 1) v = lpb[tfirst * C + blank];
        if (S >= 2 && s == S - 2) v = lpb[tfirst * C + lab[k]];
      }
      cur[s] = v;
      out[tfirst * S_max + s] = v;
    }
  }
  __syncthreads();
  for (int64_t n0 = 1; n0 < Tb; n0 += CH) {
    float em[SPT][CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int64_t n = n0 + j;
      const int64_t t = bwd ? Tb - 1 - n : n;
#pragma unroll
      for (int k = 0; k < SPT; ++k) {
        const int s = threadIdx.x + k * blockDim.x;
        em[k][j] = (n < Tb && s < S) ? lpb[t * C + lab[k]] : 0.f;
      }
    }
    float av[SPT][CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (n0 + j < Tb) {   // uniform over the block
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
          const int s = threadIdx.x + k * blockDim.x;
          av[k][j] = NEG_INF;
          if (s < S) {
            float a = cur[s];
            // branch-free: a missing predecessor enters as -inf (lse2_fast(a, -inf) == a exactly)
            if (!bwd) {
              a = lse2_fast(a, s >= 1 ? cur[s >= 1 ? s - 1 : 0] : NEG_INF);
              a = lse2_fast(a, skip[k] ? cur[s >= 2 ? s - 2 : 0] : NEG_INF);
            } else {
              a = lse2_fast(a, s + 1 < S ? cur[s + 1] : NEG_INF);
              a = lse2_fast(a, skip[k] ? cur[s + 2 < S ? s + 2 : s] : NEG_INF);
            }
            const float v = (a == NEG_INF) ? NEG_INF : a + em[k][j];
            nxt[s] = v;
            av[k][j] = v;
          }
        }
        __syncthreads();
        float* tmp = cur; cur = nxt; nxt = tmp;
      }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int64_t n = n0 + j;
      const int64_t t = bwd ? Tb - 1 - n : n;
#pragma unroll
      for (int k = 0; k < SPT; ++k) {
        const int s = threadIdx.x + k * blockDim.x;
        if (n < Tb && s < S) out[t * S_max + s] = av[k][j];
      }
    }
  }
  if (!bwd && threadIdx.x == 0) {
    float ll = cur[S - 1];
    if (S >= 2) ll = lse2(ll, cur[S - 2]);
    const float nll = -ll;
    nll_out[b] = (!(nll < INFINITY) && zero_inf) ? 0.f : nll;
  }
}

__global__ __launch_bounds__(256) void ctc_grad_kernel(const float* __restrict__ lp, const int64_t* __restrict__ targets,
                                                       const int64_t* __restrict__ in_len,
                                                       const int64_t* __restrict__ tgt_len,
                                                       const float* __restrict__ alpha, const float* __restrict__ beta,
                                                       float* __restrict__ grad, int64_t T, int C, int64_t Umax,
                                                       int blank, float scale, int zero_inf) {
  extern __shared__ float sh[];
  const int64_t b = blockIdx.x;
  const int64_t t0 = (int64_t)blockIdx.y * CTC_FPB;
  const int64_t t1 = t0 + CTC_FPB < T ? t0 + CTC_FPB : T;
  const int64_t S_max = 2 * Umax + 1;
  const int64_t U = tgt_len[b] < Umax ? tgt_len[b] : Umax;
  const int64_t S = 2 * U + 1;
  const int64_t Tb = in_len[b] < T ? in_len[b] : T;
  float* gb = grad + b * T * C;
  if (Tb <= 0) {
    for (int64_t i = t0 * C + threadIdx.x; i < t1 * C; i += blockDim.x) gb[i] = 0.f;
    return;
  }
  const float* al = alpha + b * T * S_max;
  const float* be = beta + b * T * S_max;
  float ll = al[(Tb - 1) * S_max + S - 1];
  if (S >= 2) ll = lse2(ll, al[(Tb - 1) * S_max + S - 2]);
  const float nll = -ll;
  if (!(nll < INFINITY)) {
    const float fill = zero_inf ? 0.f : NAN;
    for (int64_t i = t0 * C + threadIdx.x; i < t1 * C; i += blockDim.x) gb[i] = fill;
    return;
  }
  const int64_t tv = t1 < Tb ? t1 : Tb;    // frames of this block inside the utterance: [t0, tv)
  for (int64_t i = (t0 > tv ? t0 : tv) * C + threadIdx.x; i < t1 * C; i += blockDim.x) gb[i] = 0.f;
  if (t0 >= tv) return;
  float* contrib = sh;                                  // S_max
  int* lab = reinterpret_cast<int*>(sh + S_max);        // S_max
  int* nxt = reinterpret_cast<int*>(sh + 2 * S_max);    // S_max: next odd position with the same label
  int* head = reinterpret_cast<int*>(sh + 3 * S_max);   // C: first odd position of each label (-1: none)
  __shared__ float blank_sh;
  const float* lpb = lp + b * T * C;
  for (int64_t s = threadIdx.x; s < S; s += blockDim.x) lab[s] = ctc_label(targets + b * Umax, s, blank);
  for (int c = threadIdx.x; c < C; c += blockDim.x) head[c] = INT_MAX;
  __syncthreads();
  // per-label position lists: the posterior of class c is summed over its positions in ascending order, a
  // fixed order, so the logits gradient is bitwise reproducible.  Built in parallel: head[c] = the first odd
  // position of label c (an LDS atomic min: order-free), nxt[s] = the next odd position after s with the
  // same label (a forward scan per position) -- one thread walking all positions cost ~6 us per block
  for (int64_t s = 2 * threadIdx.x + 1; s < S; s += 2 * blockDim.x) {
    const int l = lab[s];
    if (l >= 0 && l < C) {
      atomicMin(&head[l], (int)s);
      int nx = -1;
      for (int64_t s2 = s + 2; s2 < S; s2 += 2)
        if (lab[s2] == l) {
          nx = (int)s2;
          break;
        }
      nxt[s] = nx;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    if (head[c] == INT_MAX) head[c] = -1;
  __syncthreads();
  for (int64_t t = t0; t < tv; ++t) {
    for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
      const float ab = al[t * S_max + s] + be[t * S_max + s];
      contrib[s] = (ab > NEG_INF) ? __expf(ab - lpb[t * C + lab[s]] + nll) : 0.f;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // blank posterior: the even positions, lane-strided + butterfly
      float v = 0.f;
      for (int64_t s = 2 * threadIdx.x; s < S; s += 128) v += contrib[s];
      v = wave_sum(v);
      if (threadIdx.x == 0) blank_sh = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float post = (c == blank) ? blank_sh : 0.f;
      for (int s = head[c]; s >= 0; s = nxt[s]) post += contrib[s];
      gb[t * C + c] = scale * (__expf(lpb[t * C + c]) - post);
    }
    __syncthreads();
  }
}

// grad += coef*(softmax(lp/T) - p_t) ; loss_acc += loss_scale * sum_c p_t (log p_t - log_softmax(lp/T))
// teacher p_t = softmax(log_softmax(tl)/T)   (tl: teacher decoder logits)
// Rows are strided over a fixed grid (each wave takes rows w, w + 4 gridDim, ...) and the loss partials meet
// in LDS: one float atomic per workgroup -- an atomic per row (12 832 at the bench shape, all on one address)
// serialised at the L2 and made this launch ~170 us in the step.
template <int NV>
__global__ __launch_bounds__(256) void kl_kernel(const float* __restrict__ lp, const float* __restrict__ tl,
                                                 float* __restrict__ grad, float* __restrict__ loss_acc, int64_t rows,
                                                 int C, float invT, float coef, float loss_scale) {
  const int lane = threadIdx.x & 63;
  __shared__ float wsum[4];
  float contrib = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    float sv[NV], tv[NV];
    float ms = NEG_INF, mt = NEG_INF;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      sv[i] = (c < C) ? lp[r * C + c] * invT : NEG_INF;
      tv[i] = (c < C) ? tl[r * C + c] : NEG_INF;
      ms = fmaxf(ms, sv[i]);
      mt = fmaxf(mt, tv[i]);
    }
    ms = wave_max(ms);
    mt = wave_max(mt);
    float ss = 0.f, st = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      ss += (lane + 64 * i < C) ? __expf(sv[i] - ms) : 0.f;
      st += (lane + 64 * i < C) ? __expf(tv[i] - mt) : 0.f;
    }
    const float lzs = ms + __logf(wave_sum(ss));
    const float lzt = mt + __logf(wave_sum(st));
    // teacher: logp = tl - lzt ; then q = softmax(logp / T)
    float q[NV];
    float mq = NEG_INF;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      q[i] = (lane + 64 * i < C) ? (tv[i] - lzt) * invT : NEG_INF;
      mq = fmaxf(mq, q[i]);
    }
    mq = wave_max(mq);
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) sq += (lane + 64 * i < C) ? __expf(q[i] - mq) : 0.f;
    const float lzq = mq + __logf(wave_sum(sq));
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        const float logpt = q[i] - lzq;
        const float pt = __expf(logpt);
        const float logps = sv[i] - lzs;
        if (pt > 0.f) contrib += pt * (logpt - logps);
        grad[r * C + c] += coef * (__expf(logps) - pt);
      }
    }
  }
  contrib = wave_sum(contrib);
  if (lane == 0) wsum[threadIdx.x >> 6] = contrib;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    if (t != 0.f) atomicAdd(loss_acc, t * loss_scale);
  }
}

// out = [total, ctc, kl, recon, fm] ; ctc = mean_b nll ; total = ctc + kd_alpha*kl + recon + fm
__global__ void loss_combine_kernel(const float* __restrict__ nll, int64_t B, const float* __restrict__ kl,
                                    const float* __restrict__ recon, const float* __restrict__ fm, float kd_alpha,
                                    float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float s = 0.f;
  for (int64_t b = 0; b < B; ++b) s += nll[b];
  const float ctc = s / (float)B;
  const float k = kl ? kl[0] : 0.f, r = recon ? recon[0] : 0.f, f = fm ? fm[0] : 0.f;
  out[0] = ctc + kd_alpha * k + r + f;
  out[1] = ctc;
  out[2] = k;
  out[3] = r;
  out[4] = f;
}

// values per lane of the row kernels: the smallest compiled NV with 64 * NV >= C (C <= 4096)
template <typename F>
int row_dispatch(int64_t C, F&& go) {
  if (C <= 256) return go(std::integral_constant<int, 4>{});
  if (C <= 512) return go(std::integral_constant<int, 8>{});
  if (C <= 1088) return go(std::integral_constant<int, 17>{});   // V = 1024 BPE: 1025 classes
  if (C <= 2048) return go(std::integral_constant<int, 32>{});
  return go(std::integral_constant<int, 64>{});
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_log_softmax(const float* x, float* y, int64_t rows, int64_t C, int64_t ldx, int64_t ldy, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && y, "null pointer");
  KDFM_REQUIRE(C > 0 && C <= 4096, "classes in (0,4096]");
  if (rows == 0) return KDFM_OK;
  return row_dispatch(C, [&](auto nv) {
    hipLaunchKernelGGL(log_softmax_kernel<decltype(nv)::value>, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0,
                       as_stream(stream), x, y, rows, (int)C, ldx, ldy);
    return check_launch("kdfm_log_softmax");
  });
}

int kdfm_argmax_rows(const float* x, int64_t* idx, int64_t rows, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && idx && C > 0, "bad args");
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(argmax_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream), x, idx, rows,
                     (int)C);
  return check_launch("kdfm_argmax_rows");
}

int kdfm_log_softmax_bwd(const float* dy, const float* y, float* dx, int64_t rows, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy && y && dx, "null pointer");
  KDFM_REQUIRE(C > 0 && C <= 4096, "classes in (0,4096]");
  if (rows == 0) return KDFM_OK;
  return row_dispatch(C, [&](auto nv) {
    hipLaunchKernelGGL(log_softmax_bwd_kernel<decltype(nv)::value>, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0,
                       as_stream(stream), dy, y, dx, rows, (int)C);
    return check_launch("kdfm_log_softmax_bwd");
  });
}

int kdfm_ctc_loss(const float* log_probs, const int64_t* targets, const int64_t* input_lengths,
                  const int64_t* target_lengths, float* alpha_ws, float* beta_ws, float* nll, float* grad, int64_t B,
                  int64_t T, int64_t C, int64_t Umax, int64_t blank, float grad_scale, int32_t zero_infinity,
                  void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(log_probs && targets && input_lengths && target_lengths && alpha_ws && beta_ws && nll && grad,
               "null pointer");
  KDFM_REQUIRE(blank >= 0 && blank < C && C <= 4096 && Umax >= 1 && Umax <= 4096, "bad sizes");
  if (B == 0) return KDFM_OK;
  const int64_t S_max = 2 * Umax + 1;
  const size_t sh_ab = sizeof(float) * 2 * S_max;
  const size_t sh_gr = sizeof(float) * (3 * S_max + C);
  KDFM_REQUIRE(sh_gr <= 60 * 1024, "CTC workspace exceeds LDS");
  hipStream_t st = as_stream(stream);
  const unsigned nt = S_max <= 256 ? 256 : 1024;
  const int64_t spt = ceil_div(S_max, nt);
  const dim3 gab((unsigned)B, 2);
#define KDFM_CTC_AB(SPT_, CH_)                                                                                   \
  hipLaunchKernelGGL((ctc_ab_kernel<SPT_, CH_>), gab, dim3(nt), sh_ab, st, log_probs, targets, input_lengths,  \
                     target_lengths, alpha_ws, beta_ws, nll, T, (int)C, Umax, (int)blank, zero_infinity)
  if (spt <= 1) KDFM_CTC_AB(1, 16);
  else if (spt <= 2) KDFM_CTC_AB(2, 8);
  else if (spt <= 4) KDFM_CTC_AB(4, 4);
  else KDFM_CTC_AB(9, 2);
#undef KDFM_CTC_AB
  if (int rc = check_launch("kdfm_ctc_loss (alpha/beta)")) return rc;
  if (T <= 0) return KDFM_OK;
  hipLaunchKernelGGL(ctc_grad_kernel, dim3((unsigned)B, (unsigned)ceil_div(T, CTC_FPB)), dim3(256), sh_gr, st,
                     log_probs, targets, input_lengths, target_lengths, alpha_ws, beta_ws, grad, T, (int)C, Umax,
                     (int)blank, grad_scale, zero_infinity);
  return check_launch("kdfm_ctc_loss");
}

int kdfm_kl_div_logits(const float* student_logp, const float* teacher_logits, float* grad, float* loss_acc,
                       int64_t rows, int64_t C, float temperature, float grad_coef, float loss_scale, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(student_logp && teacher_logits && grad && loss_acc, "null pointer");
  KDFM_REQUIRE(C > 0 && C <= 4096 && temperature > 0.f, "bad args");
  if (rows == 0) return KDFM_OK;
  return row_dispatch(C, [&](auto nv) {
    const int64_t nb = ceil_div(rows, 4);
    hipLaunchKernelGGL(kl_kernel<decltype(nv)::value>, dim3((unsigned)(nb < 512 ? nb : 512)), dim3(256), 0,
                       as_stream(stream), student_logp, teacher_logits, grad, loss_acc, rows, (int)C, 1.f / temperature,
                       grad_coef, loss_scale);
    return check_launch("kdfm_kl_div_logits");
  });
}

int kdfm_loss_combine(const float* nll, int64_t B, const float* kl, const float* recon, const float* fm,
                      float kd_alpha, float* out5, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(nll && out5 && B > 0, "bad args");
  hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(64), 0, as_stream(stream), nll, B, kl, recon, fm, kd_alpha,
                     out5);
  return check_launch("kdfm_loss_combine");
}

}  // extern "C"
