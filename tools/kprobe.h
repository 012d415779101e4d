// In-kernel phase probe for the tools/*_probe.hip timing tools (test tooling, not the library): every
// wave's lane 0 records the shader clock (s_memtime) at KPROBE(i) points into g_pb[wave][i] (32 slots),
// and the 100 MHz real-time clock at slots 0 and 31 for calibration.  Include BEFORE the kernel source.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ unsigned long long* g_pb;
__device__ unsigned long long* g_rt;
#define KPROBE(i)                                                                                    \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0) {                                                                   \
      const size_t w_ = ((size_t)blockIdx.x + (size_t)blockIdx.y * gridDim.x) * (blockDim.x >> 6) + \
                        (threadIdx.x >> 6);                                                          \
      g_pb[w_ * 32 + (i)] = __builtin_amdgcn_s_memtime();                                            \
      if ((i) == 0 || (i) == 31) g_rt[w_ * 2 + ((i) == 31)] = __builtin_amdgcn_s_memrealtime();      \
    }                                                                                                \
  } while (0)

struct KProbe {
  unsigned long long *pb = nullptr, *rt = nullptr;
  size_t nw = 0;
  void alloc(size_t waves) {
    nw = waves;
    (void)hipMalloc(&pb, nw * 32 * 8);
    (void)hipMalloc(&rt, nw * 2 * 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pb), &pb, sizeof(pb));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rt), &rt, sizeof(rt));
  }
  void clear() {
    (void)hipMemset(pb, 0, nw * 32 * 8);
    (void)hipMemset(rt, 0, nw * 2 * 8);
  }
  // per probe: mean cycles since probe 0 over the waves that recorded it
  void report(const char* title, float us_per_launch) {
    std::vector<unsigned long long> h(nw * 32), hr(nw * 2);
    (void)hipMemcpy(h.data(), pb, h.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hr.data(), rt, hr.size() * 8, hipMemcpyDeviceToHost);
    double sum[32] = {0}, cnt[32] = {0}, cyc = 0, rts = 0;
    for (size_t w = 0; w < nw; ++w) {
      const unsigned long long* q = &h[w * 32];
      if (!q[0]) continue;
      for (int i = 1; i < 32; ++i)
        if (q[i]) {
          sum[i] += (double)(q[i] - q[0]);
          cnt[i] += 1;
        }
      if (q[31] && hr[w * 2 + 1]) {
        cyc += (double)(q[31] - q[0]);
        rts += (double)(hr[w * 2 + 1] - hr[w * 2]);
      }
    }
    const double mhz = rts > 0 ? cyc / rts * 100.0 : 0.0;
    printf("%s: %.1f us per launch; shader clock %.0f MHz\n", title, us_per_launch, mhz);
    for (int i = 1; i < 32; ++i)
      if (cnt[i] > 0)
        printf("  probe %2d: %8.0f cycles (%6.2f us) after start, %6.0f waves\n", i, sum[i] / cnt[i],
               mhz > 0 ? sum[i] / cnt[i] / mhz : 0.0, cnt[i]);
    fflush(stdout);
  }
};
