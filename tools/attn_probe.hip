// Phase timing of the fused rel-pos attention forward (csrc/attn_fused.hip) at the bench shapes:
// per-wave shader-clock stamps at its KPROBE points (after each key block's staging, scores,
// softmax / P writes and PV), averaged over all waves.  Standalone test tool, not the library.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/attn_probe.hip \
//          -L kd-via-fm-in-asr_amd/kdfm -lkdfm -Wl,-rpath,'$ORIGIN/../kd-via-fm-in-asr_amd/kdfm' -o tools/attn_probe
#include "kprobe.h"

#include "../kd-via-fm-in-asr_amd/csrc/attn_fused.hip"

#include <cstdlib>

static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  srand(seed);
  for (auto& v : h) v = scale * ((rand() / (float)RAND_MAX) * 2.f - 1.f);
  float* d;
  (void)hipMalloc(&d, n * 4);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

static void run(int64_t B, int64_t T, int64_t d, int64_t H, float p, KProbe& kp, bool wpt = true) {
  const int64_t rows = B * T;
  float* qu = dev_rand(rows * d, 1.f, 1);
  float* qv = dev_rand(rows * d, 1.f, 2);
  float* qkv = dev_rand(rows * 3 * d, 1.f, 3);
  float* pos = dev_rand((2 * T - 1) * d, 1.f, 4);
  std::vector<int64_t> hl(B, T);
  int64_t* lens;
  (void)hipMalloc(&lens, B * 8);
  (void)hipMemcpy(lens, hl.data(), B * 8, hipMemcpyHostToDevice);
  float *o, *lse, *mblk;
  uint16_t* pt;
  (void)hipMalloc(&o, rows * d * 4);
  (void)hipMalloc(&lse, B * H * T * 4);
  (void)hipMalloc(&pt, B * H * T * T * 2);
  (void)hipMalloc(&mblk, B * H * T * ((T + 63) / 64) * 4);
  uint64_t* seed;
  (void)hipMalloc(&seed, 8);
  (void)hipMemset(seed, 7, 8);
  const float scale = 1.f / sqrtf((float)(d / H));
  auto launch = [&]() {
    if (kdfm_relpos_attn_fwd(qu, qv, qkv, pos, lens, o, nullptr, nullptr, lse, wpt ? pt : nullptr, wpt ? mblk : nullptr,
                             B, H, T, d, scale, p, seed, 5, nullptr))
      exit(3);
  };
  for (int i = 0; i < 3; ++i) launch();
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < 10; ++i) launch();
  (void)hipEventRecord(e1, nullptr);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  kp.clear();
  launch();
  (void)hipDeviceSynchronize();
  char title[128];
  snprintf(title, sizeof title, "relpos_attn_fwd B=%lld T=%lld d=%lld H=%lld p=%.1f%s", (long long)B, (long long)T,
           (long long)d, (long long)H, p, wpt ? " (p~ / m_blk)" : " (lse only: the bench's bwd2 mode)");
  kp.report(title, 1e3f * ms / 10);
  (void)hipFree(qu); (void)hipFree(qv); (void)hipFree(qkv); (void)hipFree(pos); (void)hipFree(lens);
  (void)hipFree(o); (void)hipFree(lse); (void)hipFree(pt); (void)hipFree(mblk); (void)hipFree(seed);
}

int main() {
  KProbe kp;
  kp.alloc((size_t)7 * 32 * 8 * 4);
  run(32, 401, 176, 4, 0.1f, kp, false);
  run(32, 401, 176, 4, 0.0f, kp, false);
  run(32, 401, 512, 8, 0.1f, kp, false);
  return 0;
}
