// Evaluation path: CTC greedy decoding on the device and the word-level
// Levenshtein distance of the WER metric on the host.
//
//   kdfm_ctc_greedy: NeMo CTC 'greedy' decoding as used by WER.update (metrics/wer.py:329-333;
//     semantics SURVEY.md Appendix A.9): per utterance, argmax over the C classes of every valid
//     frame (first index on ties = torch.argmax), collapse repeats, drop the blank, compact left.
//     One workgroup per utterance: waves take frames (lanes over classes, wave argmax), the per-frame
//     labels go to LDS, then 256 threads compact their frame slices with a block prefix count.
//   kdfm_edit_distance: editdistance.eval (wer.py:66-69, 351) on integer-coded tokens.
#include <vector>

#include "common.h"

namespace kdfm {
namespace {

constexpr int GD_NT = 256;

__global__ __launch_bounds__(GD_NT) void ctc_greedy_kernel(const float* __restrict__ lp, int64_t ld,
                                                           const int64_t* __restrict__ lens, int32_t* __restrict__ tok,
                                                           int32_t* __restrict__ ntok, int32_t* __restrict__ labels,
                                                           int T, int C, int blank, int fold) {
  extern __shared__ int am[];  // T per-frame labels, then GD_NT counts
  int* cnt = am + T;
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int len = lens ? (int)lens[b] : T;
  len = len < 0 ? 0 : (len > T ? T : len);
  for (int t = w; t < len; t += GD_NT / 64) {
    const float* row = lp + ((int64_t)b * T + t) * ld;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float v = row[c];
      if (v > best) { best = v; bi = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) am[t] = (bi == 0x7fffffff) ? 0 : bi;
  }
  __syncthreads();
  // contiguous frame slice per thread; a frame is kept when it is not blank and (fold) differs
  // from the previous frame's label (blanks included: "a _ a" keeps both a's)
  const int per = (len + GD_NT - 1) / GD_NT;
  const int t0 = threadIdx.x * per, t1 = min(t0 + per, len);
  int n = 0;
  for (int t = t0; t < t1; ++t) {
    const int a = am[t];
    if (a != blank && (!fold || t == 0 || am[t - 1] != a)) ++n;
  }
  cnt[threadIdx.x] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < GD_NT; ++i) {
      const int c = cnt[i];
      cnt[i] = s;
      s += c;
    }
    ntok[b] = s;
  }
  __syncthreads();
  int pos = cnt[threadIdx.x];
  for (int t = t0; t < t1; ++t) {
    const int a = am[t];
    if (a != blank && (!fold || t == 0 || am[t - 1] != a)) tok[(int64_t)b * T + pos++] = a;
  }
  if (labels)
    for (int t = threadIdx.x; t < T; t += GD_NT) labels[(int64_t)b * T + t] = (t < len) ? am[t] : blank;
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_ctc_greedy(const float* log_probs, int64_t ld, const int64_t* lengths, int32_t* tokens, int32_t* ntok,
                    int32_t* labels, int64_t B, int64_t T, int64_t C, int64_t blank, int32_t fold, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(log_probs && tokens && ntok, "null pointer");
  KDFM_REQUIRE(B >= 0 && T > 0 && T <= 16384 && C > 0 && ld >= C, "bad shape");
  KDFM_REQUIRE(blank >= 0 && blank < C, "blank out of range");
  if (B == 0) return KDFM_OK;
  const size_t lds = (size_t)(T + GD_NT) * sizeof(int);
  hipLaunchKernelGGL(ctc_greedy_kernel, dim3((unsigned)B), dim3(GD_NT), lds, as_stream(stream), log_probs, ld, lengths,
                     tokens, ntok, labels, (int)T, (int)C, (int)blank, (int)fold);
  return check_launch("kdfm_ctc_greedy");
}

int64_t kdfm_edit_distance(const int32_t* a, int64_t na, const int32_t* b, int64_t nb) {
  if (na < 0 || nb < 0 || (na > 0 && !a) || (nb > 0 && !b)) return -1;
  if (na == 0) return nb;
  if (nb == 0) return na;
  std::vector<int64_t> prev((size_t)nb + 1), cur((size_t)nb + 1);
  for (int64_t j = 0; j <= nb; ++j) prev[(size_t)j] = j;
  for (int64_t i = 1; i <= na; ++i) {
    cur[0] = i;
    for (int64_t j = 1; j <= nb; ++j) {
      const int64_t sub = prev[(size_t)j - 1] + (a[i - 1] != b[j - 1] ? 1 : 0);
      const int64_t del = prev[(size_t)j] + 1, ins = cur[(size_t)j - 1] + 1;
      cur[(size_t)j] = sub < del ? (sub < ins ? sub : ins) : (del < ins ? del : ins);
    }
    prev.swap(cur);
  }
  return prev[(size_t)nb];
}

}  // extern "C"
