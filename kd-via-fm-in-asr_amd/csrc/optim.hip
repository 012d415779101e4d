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

// p16 (nullable): the updated parameters also written as bf16 (round to nearest even) into a mirror of the flat
// buffer -- the large-tile GEMM's weight operands (kdfm_adamw_noam_bf16), so no per-weight cast per step
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    const int64_t* __restrict__ step,
                                                    int64_t* __restrict__ adam_base, float base, float d_model,
                                                    float warmup, float min_lr, float b1, float b2, float eps, float wd,
                                                    float gscale, float* __restrict__ lr_out,
                                                    const float* __restrict__ gstats, uint16_t* __restrict__ p16) {
  const int64_t k = step[0];
  const float lr = noam_lr(k, base, d_model, warmup, min_lr);
  if (lr_out && blockIdx.x == 0 && threadIdx.x == 0) lr_out[0] = lr;
  if (gstats && gstats[1] != 0.f) {
    // a non-finite gradient: parameters and moments unchanged.  The schedule still advances (Lightning
    // steps the scheduler after a skipped optimizer step) but AdamW's own step count does not (torch only
    // counts steps that update the moments): the moments' origin moves one step later
    if (adam_base && blockIdx.x == 0 && threadIdx.x == 0) adam_base[0] += 1;
    return;
  }
  const int64_t ka = adam_base ? k - adam_base[0] : k;   // AdamW's own step count
  const float bc1 = 1.f - powf(b1, (float)ka);
  const float bc2 = 1.f - powf(b2, (float)ka);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  auto upd = [&](float& pi, float gi, float& mi, float& vi) {
    gi *= gscale;
    pi *= (1.f - lr * wd);
    mi = b1 * mi + (1.f - b1) * gi;
    vi = b2 * vi + (1.f - b2) * gi * gi;
    pi -= step_size * mi / (sqrtf(vi) / bc2s + eps);
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  // 16-byte lanes when the four buffers are aligned (the flat parameter buffer is): the same per-element update
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                   (((uintptr_t)p16) & 7) == 0;
  const int64_t n4 = vec ? n / 4 : 0;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[q], mm = reinterpret_cast<float4*>(m)[q];
    float4 vv = reinterpret_cast<float4*>(v)[q];
    const float4 gg = reinterpret_cast<const float4*>(g)[q];
    upd(pp.x, gg.x, mm.x, vv.x);
    upd(pp.y, gg.y, mm.y, vv.y);
    upd(pp.z, gg.z, mm.z, vv.z);
    upd(pp.w, gg.w, mm.w, vv.w);
    reinterpret_cast<float4*>(m)[q] = mm;
    reinterpret_cast<float4*>(v)[q] = vv;
    reinterpret_cast<float4*>(p)[q] = pp;
    if (p16) reinterpret_cast<uint2*>(p16)[q] = make_uint2(pack_bf16x2(pp.x, pp.y), pack_bf16x2(pp.z, pp.w));
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float pi = p[i], mi = m[i], vi = v[i];
    upd(pi, g[i], mi, vi);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (p16) p16[i] = f2bf(pi);
  }
}

// gradient statistics: per-workgroup partials of sum g^2 and of the non-finite count over a fixed
// grid (grid-stride, fixed lane order), then one workgroup folds them in a fixed tree: deterministic
constexpr int GS_BLOCKS = 512;

__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  a = red[0] + red[2] + (red[4] + red[6]);
  b = red[1] + red[3] + (red[5] + red[7]);
}

__global__ __launch_bounds__(256) void grad_stats_kernel(const float* __restrict__ g, int64_t n, float scale,
                                                         float* __restrict__ part) {
  __shared__ float red[8];
  float ss = 0.f, bad = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  const bool vec = (((uintptr_t)g) & 15) == 0;
  for (int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i0 < n; i0 += stride) {
    float v[4];
    if (vec && i0 + 4 <= n) {
      const float4 q = *reinterpret_cast<const float4*>(g + i0);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = i0 + e < n ? g[i0 + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = v[e] * scale;
      if (isfinite(x)) ss += x * x; else bad += 1.f;
    }
  }
  block_sum2(ss, bad, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ss;
    part[2 * blockIdx.x + 1] = bad;
  }
}

__global__ __launch_bounds__(256) void grad_stats_fold_kernel(const float* __restrict__ part, int nb,
                                                              float* __restrict__ out) {
  __shared__ float red[8];
  float ss = 0.f, bad = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) {
    ss += part[2 * i];
    bad += part[2 * i + 1];
  }
  block_sum2(ss, bad, red);
  if (threadIdx.x == 0) {
    out[0] = ss;
    out[1] = bad;
  }
}

}  // namespace
}  // namespace kdfm

extern "C" int64_t kdfm_grad_stats_ws(void) { return 2 * kdfm::GS_BLOCKS; }

extern "C" int kdfm_grad_stats(const float* grads, int64_t n, float scale, float* ws, int64_t ws_len, float* out2,
                               void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(grads && ws && out2 && n >= 0, "bad args");
  KDFM_REQUIRE(ws_len >= 2 * GS_BLOCKS, "workspace too small (kdfm_grad_stats_ws)");
  int64_t nb = ceil_div(n, 1024);
  if (nb > GS_BLOCKS) nb = GS_BLOCKS;
  if (nb < 1) nb = 1;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(grad_stats_kernel, dim3((unsigned)nb), dim3(256), 0, st, grads, n, scale, ws);
  int rc = check_launch("kdfm_grad_stats");
  if (rc) return rc;
  hipLaunchKernelGGL(grad_stats_fold_kernel, dim3(1), dim3(256), 0, st, ws, (int)nb, out2);
  return check_launch("kdfm_grad_stats(fold)");
}

extern "C" int kdfm_adamw_noam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                               const int64_t* step, int64_t* adam_base, float base_lr, float d_model, float warmup_steps, float min_lr,
                               float beta1, float beta2, float eps, float weight_decay, float grad_scale,
                               float* lr_out, const float* gstats, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(params && grads && exp_avg && exp_avg_sq && step, "null pointer");
  if (n == 0) return KDFM_OK;
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), params, grads, exp_avg,
                     exp_avg_sq, n, step, adam_base, base_lr, d_model, warmup_steps, min_lr, beta1, beta2, eps, weight_decay,
                     grad_scale, lr_out, gstats, (uint16_t*)nullptr);
  return check_launch("kdfm_adamw_noam");
}

extern "C" int kdfm_adamw_noam_bf16(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                                    uint16_t* params_bf16, int64_t n, const int64_t* step, int64_t* adam_base,
                                    float base_lr, float d_model, float warmup_steps, float min_lr, float beta1,
                                    float beta2, float eps, float weight_decay, float grad_scale, float* lr_out,
                                    const float* gstats, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(params && grads && exp_avg && exp_avg_sq && step && params_bf16, "null pointer");
  if (n == 0) return KDFM_OK;
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), params, grads, exp_avg,
                     exp_avg_sq, n, step, adam_base, base_lr, d_model, warmup_steps, min_lr, beta1, beta2, eps, weight_decay,
                     grad_scale, lr_out, gstats, params_bf16);
  return check_launch("kdfm_adamw_noam_bf16");
}
