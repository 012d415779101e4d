// Output-side losses of the ver5 step:
//   log_softmax of the ConvASRDecoder logits (conv_asr.py:456-468),
//   CTC (NeMo CTCLoss -> torch CTCLoss, losses/ctc.py:68-82; blank = V, zero_infinity, mean_batch
//   from ctc_models.py:81-85) with its logits gradient exp(lp) - posterior,
//   logit KD (asr_train_diffm.py:751-756: kl_div(log_softmax(s/T), softmax(t/T), 'batchmean') * T^2),
//   and the final loss assembly (asr_train_diffm.py:803-811).
#include <math.h>

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

__global__ __launch_bounds__(256) void log_softmax_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t rows,
                                                          int C, int64_t ldx, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float v[4];
  float mx = NEG_INF;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < C) ? x[r * ldx + c] : NEG_INF;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += (lane + 64 * i < C) ? __expf(v[i] - mx) : 0.f;
  const float lz = mx + __logf(wave_sum(s));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
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
__global__ __launch_bounds__(256) void log_softmax_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                              float* __restrict__ dx, int64_t rows, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float g[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    g[i] = (c < C) ? dy[r * C + c] : 0.f;
    s += g[i];
  }
  s = wave_sum(s);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < C) dx[r * C + c] = g[i] - __expf(y[r * C + c]) * s;
  }
}

// One block per utterance.  alpha/beta workspaces (B, T, S) in log space; nll (B);
// grad (B, T, C) = scale * (exp(lp) - posterior) for t < len, 0 beyond (or all 0 if infeasible).
__global__ __launch_bounds__(256) void ctc_kernel(const float* __restrict__ lp, const int64_t* __restrict__ targets,
                                                  const int64_t* __restrict__ in_len, const int64_t* __restrict__ tgt_len,
                                                  float* __restrict__ alpha, float* __restrict__ beta,
                                                  float* __restrict__ nll_out, float* __restrict__ grad, int64_t T,
                                                  int C, int64_t Umax, int blank, float scale, int zero_inf) {
  extern __shared__ float sh[];
  const int64_t b = blockIdx.x;
  const int64_t S_max = 2 * Umax + 1;
  const int64_t U = tgt_len[b] < Umax ? tgt_len[b] : Umax;
  const int64_t S = 2 * U + 1;
  int64_t Tb = in_len[b] < T ? in_len[b] : T;
  float* prev = sh;                      // S_max
  float* cur = sh + S_max;               // S_max
  int* lab = reinterpret_cast<int*>(sh + 2 * S_max);  // S_max
  float* contrib = sh + 3 * S_max;       // S_max: per-position posterior term of the current frame
  int* nxt = reinterpret_cast<int*>(sh + 4 * S_max);  // S_max: next odd position with the same label
  int* head = reinterpret_cast<int*>(sh + 5 * S_max);  // C: first odd position of each label (-1: none)
  __shared__ float nll_sh, blank_sh;
  const float* lpb = lp + b * T * C;
  float* al = alpha + b * T * S_max;
  float* be = beta + b * T * S_max;
  for (int64_t s = threadIdx.x; s < S; s += blockDim.x)
    lab[s] = (s & 1) ? (int)targets[b * Umax + (s >> 1)] : blank;
  __syncthreads();
  // per-label position lists (built once per utterance by one lane): the posterior of class c at a
  // frame is summed over its positions in ascending order, a fixed order (no LDS atomics), so the
  // logits gradient is bitwise reproducible
  if (threadIdx.x == 0) {
    for (int c = 0; c < C; ++c) head[c] = -1;
    for (int64_t s = S - 2; s >= 1; s -= 2) {  // S = 2U+1: the odd (label) positions
      const int l = lab[s];
      if (l >= 0 && l < C) {
        nxt[s] = head[l];
        head[l] = (int)s;
      }
    }
  }
  __syncthreads();
  if (Tb <= 0) {
    if (threadIdx.x == 0) nll_out[b] = (U == 0 || !zero_inf) ? (U == 0 ? 0.f : INFINITY) : 0.f;
    for (int64_t i = threadIdx.x; i < T * C; i += blockDim.x) grad[b * T * C + i] = 0.f;
    return;
  }
  // ---- alpha ----
  for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
    float v = NEG_INF;
    if (s == 0) v = lpb[blank];
    if (s == 1) v = lpb[lab[1]];
    prev[s] = v;
    al[s] = v;
  }
  __syncthreads();
  for (int64_t t = 1; t < Tb; ++t) {
    for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
      float a = prev[s];
      if (s >= 1) a = lse2(a, prev[s - 1]);
      if (s >= 2 && lab[s] != blank && lab[s] != lab[s - 2]) a = lse2(a, prev[s - 2]);
      const float v = (a == NEG_INF) ? NEG_INF : a + lpb[t * C + lab[s]];
      cur[s] = v;
      al[t * S_max + s] = v;
    }
    __syncthreads();
    float* tmp = prev; prev = cur; cur = tmp;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float ll = prev[S - 1];
    if (S >= 2) ll = lse2(ll, prev[S - 2]);
    nll_sh = -ll;
  }
  __syncthreads();
  const float nll = nll_sh;
  const bool infeasible = !(nll < INFINITY);
  if (threadIdx.x == 0) nll_out[b] = (infeasible && zero_inf) ? 0.f : nll;
  if (infeasible) {
    const float fill = zero_inf ? 0.f : NAN;
    for (int64_t i = threadIdx.x; i < T * C; i += blockDim.x) grad[b * T * C + i] = fill;
    return;
  }
  // ---- beta + gradient, walking t backwards ----
  for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
    float v = NEG_INF;
    if (s == S - 1) v = lpb[(Tb - 1) * C + blank];
    if (S >= 2 && s == S - 2) v = lpb[(Tb - 1) * C + lab[S - 2]];
    prev[s] = v;
    be[(Tb - 1) * S_max + s] = v;
  }
  __syncthreads();
  for (int64_t t = Tb - 1; t >= 0; --t) {
    if (t < Tb - 1) {
      for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
        float a = prev[s];
        if (s + 1 < S) a = lse2(a, prev[s + 1]);
        if (s + 2 < S && lab[s] != blank && lab[s] != lab[s + 2]) a = lse2(a, prev[s + 2]);
        const float v = (a == NEG_INF) ? NEG_INF : a + lpb[t * C + lab[s]];
        cur[s] = v;
        be[t * S_max + s] = v;
      }
      __syncthreads();
      float* tmp = prev; prev = cur; cur = tmp;
    }
    for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
      const float ab = al[t * S_max + s] + prev[s];
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
      grad[(b * T + t) * C + c] = scale * (__expf(lpb[t * C + c]) - post);
    }
    __syncthreads();
  }
  for (int64_t i = Tb * C + threadIdx.x; i < T * C; i += blockDim.x) grad[b * T * C + i] = 0.f;
}

// grad += coef*(softmax(lp/T) - p_t) ; loss_acc += loss_scale * sum_c p_t (log p_t - log_softmax(lp/T))
// teacher p_t = softmax(log_softmax(tl)/T)   (tl: teacher decoder logits)
__global__ __launch_bounds__(256) void kl_kernel(const float* __restrict__ lp, const float* __restrict__ tl,
                                                 float* __restrict__ grad, float* __restrict__ loss_acc, int64_t rows,
                                                 int C, float invT, float coef, float loss_scale) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  float contrib = 0.f;
  if (r < rows) {
    float sv[4], tv[4];
    float ms = NEG_INF, mt = NEG_INF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
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
    for (int i = 0; i < 4; ++i) {
      ss += (lane + 64 * i < C) ? __expf(sv[i] - ms) : 0.f;
      st += (lane + 64 * i < C) ? __expf(tv[i] - mt) : 0.f;
    }
    const float lzs = ms + __logf(wave_sum(ss));
    const float lzt = mt + __logf(wave_sum(st));
    // teacher: logp = tl - lzt ; then q = softmax(logp / T)
    float q[4];
    float mq = NEG_INF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      q[i] = (lane + 64 * i < C) ? (tv[i] - lzt) * invT : NEG_INF;
      mq = fmaxf(mq, q[i]);
    }
    mq = wave_max(mq);
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) sq += (lane + 64 * i < C) ? __expf(q[i] - mq) : 0.f;
    const float lzq = mq + __logf(wave_sum(sq));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
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
  if (lane == 0 && r < rows) atomicAdd(loss_acc, contrib * loss_scale);
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

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_log_softmax(const float* x, float* y, int64_t rows, int64_t C, int64_t ldx, int64_t ldy, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && y, "null pointer");
  KDFM_REQUIRE(C > 0 && C <= 256, "classes in (0,256]");
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(log_softmax_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream), x, y,
                     rows, (int)C, ldx, ldy);
  return check_launch("kdfm_log_softmax");
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
  KDFM_REQUIRE(C > 0 && C <= 256, "classes in (0,256]");
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(log_softmax_bwd_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream), dy, y,
                     dx, rows, (int)C);
  return check_launch("kdfm_log_softmax_bwd");
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
  const size_t shmem = sizeof(float) * (5 * (2 * Umax + 1) + C);
  KDFM_REQUIRE(shmem <= 60 * 1024, "CTC workspace exceeds LDS");
  hipLaunchKernelGGL(ctc_kernel, dim3((unsigned)B), dim3(256), shmem, as_stream(stream), log_probs, targets,
                     input_lengths, target_lengths, alpha_ws, beta_ws, nll, grad, T, (int)C, Umax, (int)blank,
                     grad_scale, zero_infinity);
  return check_launch("kdfm_ctc_loss");
}

int kdfm_kl_div_logits(const float* student_logp, const float* teacher_logits, float* grad, float* loss_acc,
                       int64_t rows, int64_t C, float temperature, float grad_coef, float loss_scale, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(student_logp && teacher_logits && grad && loss_acc, "null pointer");
  KDFM_REQUIRE(C > 0 && C <= 256 && temperature > 0.f, "bad args");
  if (rows == 0) return KDFM_OK;
  hipLaunchKernelGGL(kl_kernel, dim3((unsigned)ceil_div(rows, 4)), dim3(256), 0, as_stream(stream), student_logp,
                     teacher_logits, grad, loss_acc, rows, (int)C, 1.f / temperature, grad_coef, loss_scale);
  return check_launch("kdfm_kl_div_logits");
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
