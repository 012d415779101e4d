// All weight images of a model in one launch per training step (kdfm_wimg_prep_batch): a job table
// (device memory, built once by the host) lists every image of the fused Conformer kernels — FFN
// chunk images, LN-projection images, row-streaming images — with the first global thread of each
// job; a thread finds its job by binary search and writes one lane's 16 bytes of one fragment.
// Replaces ~10 prep launches per layer (~300 per step) on the issuing streams.
#include "lnblock.h"
#include "wimg.h"

namespace kdfm {
namespace {

__global__ __launch_bounds__(256) void wimg_batch_kernel(const kdfm_wimg_job* __restrict__ jobs, int njobs,
                                                         int64_t total) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {   // last job with start <= g
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].start <= g) lo = mid; else hi = mid - 1;
  }
  const kdfm_wimg_job J = jobs[lo];
  const int64_t local = g - J.start;
  const int lane = (int)(local & 63);
  const int64_t f_all = local >> 6;
  int KS1 = 0, DT = 0;
  lnb::ln_dims(J.d, KS1, DT);
  float v[8];
  int64_t out;
  if (J.type == wimg::JOB_FFN) {
    const int CS = 4 * DT + 2 * KS1;
    const int nfr = J.flag ? 2 * DT + KS1 : CS;
    const int64_t c = f_all / nfr;
    const int f = (int)(f_all - c * nfr);
    wimg::ffn_frag(J.W1, J.W2, (int)J.d, (int)J.ff, KS1, DT, c, f, lane, v);
    out = (c * CS + f) * 64 + lane;
  } else if (J.type == wimg::JOB_LNPROJ) {
    wimg::lnproj_frag(J.W1, (int)J.d, KS1, DT, (int)J.kind, (int)J.flag, (int)f_all, lane, v);
    out = f_all * 64 + lane;
  } else {
    wimg::rowgemm_frag(J.W1, (int)J.d, KS1, (int)J.flag, (int)f_all, lane, v);
    out = f_all * 64 + lane;
  }
  *reinterpret_cast<bf16x8*>(J.img + out * 8) = pack_bf16x8<bf16x8>(v);
}

}  // namespace
}  // namespace kdfm

extern "C" int64_t kdfm_wimg_job_threads(const kdfm_wimg_job* j) {
  using namespace kdfm;
  int KS1, DT;
  if (!j || lnb::ln_dims(j->d, KS1, DT) != 0) return -1;
  if (j->type == wimg::JOB_FFN) {
    if (j->ff <= 0 || j->ff % 32) return -1;
    return (j->ff / 32) * (int64_t)(j->flag ? 2 * DT + KS1 : 4 * DT + 2 * KS1) * 64;
  }
  if (j->type == wimg::JOB_LNPROJ) {
    const int64_t e = kdfm_lnproj_img_elems((int32_t)j->kind, j->d, (int32_t)j->flag);
    return e > 0 ? e / 8 : -1;
  }
  if (j->type == wimg::JOB_ROWGEMM) return (int64_t)DT * KS1 * 64;
  return -1;
}

extern "C" int kdfm_wimg_prep_batch(const kdfm_wimg_job* jobs, int32_t njobs, int64_t total_threads, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(jobs && njobs > 0 && total_threads > 0, "empty job table");
  hipLaunchKernelGGL(wimg_batch_kernel, dim3((unsigned)ceil_div(total_threads, 256)), dim3(256), 0, as_stream(stream),
                     jobs, njobs, total_threads);
  return check_launch("kdfm_wimg_prep_batch");
}
