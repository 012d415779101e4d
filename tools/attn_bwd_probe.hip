// Phase timing of the attention backward dQ kernel (csrc/attn_bwd.hip) at the student bench shape:
// the forward (libkdfm) provides lse / p~ / m_blk, then per-wave shader-clock stamps at the dQ kernel's
// KPROBE points (each key block: staging, score recompute, dP / dS, dQ products).  Test tool only.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/attn_bwd_probe.hip \
//          -L kd-via-fm-in-asr_amd/kdfm -lkdfm -Wl,-rpath,'$ORIGIN/../kd-via-fm-in-asr_amd/kdfm' -o tools/attn_bwd_probe
#include "kprobe.h"

#include "../kd-via-fm-in-asr_amd/csrc/attn_bwd.hip"

#include <cmath>
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

static void run(int64_t B, int64_t T, int64_t d, int64_t H, KProbe& kp, bool v2) {
  const int64_t rows = B * T;
  float* qu = dev_rand(rows * d, 1.f, 1);
  float* qv = dev_rand(rows * d, 1.f, 2);
  float* qkv = dev_rand(rows * 3 * d, 1.f, 3);
  float* pos = dev_rand((2 * T - 1) * d, 1.f, 4);
  float* dO = dev_rand(rows * d, 1.f, 5);
  std::vector<int64_t> hl(B, T);
  int64_t* lens;
  (void)hipMalloc(&lens, B * 8);
  (void)hipMemcpy(lens, hl.data(), B * 8, hipMemcpyHostToDevice);
  float *o, *lse, *mblk, *dqu, *dqv, *ws;
  uint16_t* pt;
  (void)hipMalloc(&o, rows * d * 4);
  (void)hipMalloc(&dqu, rows * d * 4);
  (void)hipMalloc(&dqv, rows * d * 4);
  (void)hipMalloc(&lse, B * H * T * 4);
  (void)hipMalloc(&pt, B * H * T * T * 2);
  (void)hipMalloc(&mblk, B * H * T * ((T + 63) / 64) * 4);
  const int64_t wsl = kdfm_relpos_attn_bwd_ws(B, H, T, d);
  (void)hipMalloc(&ws, wsl * 4);
  uint64_t* seed;
  (void)hipMalloc(&seed, 8);
  (void)hipMemset(seed, 7, 8);
  const float scale = 1.f / sqrtf((float)(d / H));
  if (kdfm_relpos_attn_fwd(qu, qv, qkv, pos, lens, o, nullptr, nullptr, lse, pt, mblk, B, H, T, d, scale, 0.1f, seed, 5,
                           nullptr))
    exit(3);
  if (kdfm_relpos_attn_bwd_parts(dO, o, qu, qv, qkv, pos, lse, pt, mblk, lens, dqu, dqv, nullptr, nullptr, ws, wsl, B, H,
                                 T, d, scale, 0.1f, seed, 5, KDFM_ATTN_BWD_ROWDOT, nullptr))
    exit(4);
  const int64_t ldt = kdfm_relpos_attn_bwd2_ldt(T);
  uint16_t *ds2, *pd2;
  (void)hipMalloc(&ds2, B * H * T * ldt * 2);
  (void)hipMalloc(&pd2, B * H * T * ldt * 2);
  auto launch = [&]() {
    if (v2) {
      if (kdfm_relpos_attn_bwd2_dq(dO, o, qu, qv, qkv, pos, lse, lens, nullptr, ds2, pd2, dqu, dqv, B, H, T, d, scale,
                                   0.1f, seed, 5, nullptr))
        exit(6);
      return;
    }
    if (kdfm_relpos_attn_bwd_parts(dO, o, qu, qv, qkv, pos, lse, pt, mblk, lens, dqu, dqv, nullptr, nullptr, ws, wsl, B,
                                   H, T, d, scale, 0.1f, seed, 5, KDFM_ATTN_BWD_DQ, nullptr))
      exit(5);
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
  snprintf(title, sizeof title, "attn_bwd%s_dq B=%lld T=%lld d=%lld H=%lld", v2 ? "2" : "", (long long)B, (long long)T, (long long)d,
           (long long)H);
  (void)v2;
  kp.report(title, 1e3f * ms / 10);
}

int main() {
  KProbe kp;
  kp.alloc((size_t)7 * 32 * 2 * 4);
  run(32, 401, 88, 2, kp, false);
  run(32, 401, 88, 2, kp, true);
  run(1, 401, 88, 2, kp, true);
  return 0;
}
