// Fused AdamW + NoamAnnealing over the flat trainable-parameter buffer.
// Optimizer/schedule the reference gets from the teacher's .nemo config through
// ModelPT.setup_optimization (NeMo/nemo/core/classes/modelPT.py:650-897) and
// NoamAnnealing (NeMo/nemo/core/optim/lr_scheduler.py:473-530):
//   lr(s) = base * d^-0.5 * min(s^-0.5, s * warmup^-1.5), floored at min_lr after warmup,
//   s = max(1, last_epoch) where Lightning steps the scheduler after each optimizer step, so
//   optimizer step k (1-based) runs with s = max(1, k-1).
// torch.optim.AdamW semantics (decoupled decay, bias correction).  The bias correction counts the
// steps since the moments (re)started, k - adam_base: torch keeps AdamW's `step` in the optimizer
// state, so a resume that cannot restore the moments restarts it while the schedule continues.  Gradients arrive summed over
// data-parallel ranks; grad_scale = 1/world turns the sum into DDP's mean.
#include "common.h"

namespace kdfm {
namespace {

__device__ __forceinline__ float noam_lr(int64_t k, float base, float d_model, float warmup, float min_lr) {
  const double s = (double)((k - 1) > 1 ? (k - 1) : 1);
  double mult = 1.0 / sqrt((double)d_model);
  if (warmup > 0.f)
    mult *= fmin(1.0 / sqrt(s), s * pow((double)warmup, -1.5));
  else
    mult *= 1.0 / sqrt(s);
  double lr = base * mult;
  if (s > warmup && lr < min_lr) lr = min_lr;
  return (float)lr;
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    const int64_t* __restrict__ step,
                                                    const int64_t* __restrict__ adam_base, float base, float d_model,
                                                    float warmup, float min_lr, float b1, float b2, float eps, float wd,
                                                    float gscale, float* __restrict__ lr_out) {
  const int64_t k = step[0];
  const float lr = noam_lr(k, base, d_model, warmup, min_lr);
  const int64_t ka = adam_base ? k - adam_base[0] : k;   // AdamW's own step count
  const float bc1 = 1.f - powf(b1, (float)ka);
  const float bc2 = 1.f - powf(b2, (float)ka);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  if (lr_out && blockIdx.x == 0 && threadIdx.x == 0) lr_out[0] = lr;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float gi = g[i] * gscale;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step_size * mi / (sqrtf(vi) / bc2s + eps);
    p[i] = pi;
  }
}

}  // namespace
}  // namespace kdfm

extern "C" int kdfm_adamw_noam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                               const int64_t* step, const int64_t* adam_base, float base_lr, float d_model, float warmup_steps, float min_lr,
                               float beta1, float beta2, float eps, float weight_decay, float grad_scale,
                               float* lr_out, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(params && grads && exp_avg && exp_avg_sq && step, "null pointer");
  if (n == 0) return KDFM_OK;
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), params, grads, exp_avg,
                     exp_avg_sq, n, step, adam_base, base_lr, d_model, warmup_steps, min_lr, beta1, beta2, eps, weight_decay,
                     grad_scale, lr_out);
  return check_launch("kdfm_adamw_noam");
}
