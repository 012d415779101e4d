// Phase timing of the one-kernel striding subsampling forward (csrc/ssfused.hip) at the bench shape
// (B = 32, 16 s): per-wave shader-clock stamps at its KPROBE points (mel patch, conv1 operand, then per
// 32-channel chunk: conv1 computed, slab / y1 barrier, conv2 taps), averaged over all waves.
// Standalone test tool, not the library.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/ss_probe.hip \
//          -L kd-via-fm-in-asr_amd/kdfm -lkdfm -Wl,-rpath,'$ORIGIN/../kd-via-fm-in-asr_amd/kdfm' -o tools/ss_probe
#include "kprobe.h"

#include "../kd-via-fm-in-asr_amd/csrc/ssfused.hip"

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

static void run(int64_t C, bool side, KProbe& kp) {
  const int64_t B = 32, Tm = 1601, F = 80;
  const int64_t T1 = (Tm - 1) / 2 + 1, F1 = (F - 1) / 2 + 1, T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  float* mel = dev_rand(B * Tm * F, 1.f, 1);
  float* w0 = dev_rand(C * 9, 0.3f, 2);
  float* w2 = dev_rand(C * C * 9, 0.05f, 3);
  float* b0 = dev_rand(C, 0.1f, 4);
  float* b2 = dev_rand(C, 0.1f, 5);
  uint16_t* wp;
  (void)hipMalloc(&wp, kdfm_subsample_fused_wprep_elems(C) * 2);
  if (kdfm_subsample_fused_wprep(w0, w2, wp, C, nullptr)) exit(3);
  float* y2;
  (void)hipMalloc(&y2, B * T2 * F2 * C * 4);
  uint16_t* y1 = nullptr;
  if (side) (void)hipMalloc(&y1, B * T1 * F1 * C * 2);
  auto launch = [&]() {
    if (kdfm_subsample_fused(mel, nullptr, nullptr, nullptr, wp, b0, b2, y2, y1, B, Tm, F, C, nullptr)) exit(3);
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
  snprintf(title, sizeof title, "ss_fused C=%lld%s", (long long)C, side ? " (+ y1 side output)" : "");
  kp.report(title, 1e3f * ms / 10);
  (void)hipFree(mel); (void)hipFree(w0); (void)hipFree(w2); (void)hipFree(b0); (void)hipFree(b2);
  (void)hipFree(wp); (void)hipFree(y2);
  if (y1) (void)hipFree(y1);
}

int main() {
  KProbe kp;
  kp.alloc((size_t)32 * 51 * 8);
  run(88, true, kp);
  run(176, false, kp);
  return 0;
}
