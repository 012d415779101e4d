// Phase timing of the fused FFN forward kernel (csrc/ffn.hip) from inside the kernel: every wave's
// lane 0 records the shader clock at the FFN_PROBE points (prologue, first stage, each chunk
// iteration's compute end and barrier, reduction, epilogue); the host prints per-phase cycles
// averaged over all waves, and the 100 MHz real-time clock calibrates cycles to microseconds.
// Standalone test tool, not part of the library.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/ffn_probe.hip \
//          -L kd-via-fm-in-asr_amd/kdfm -lkdfm -Wl,-rpath,'$ORIGIN/../kd-via-fm-in-asr_amd/kdfm' -o tools/ffn_probe
#include <hip/hip_runtime.h>

__device__ unsigned long long* g_pb;
__device__ unsigned long long* g_rt;
#define FFN_PROBE(i)                                                                          \
  do {                                                                                        \
    if ((threadIdx.x & 63) == 0) {                                                            \
      const size_t w_ = (size_t)blockIdx.x * 16 + (threadIdx.x >> 6);                        \
      g_pb[w_ * 32 + (i)] = __builtin_amdgcn_s_memtime();                                     \
      if ((i) == 0 || (i) == 31) g_rt[w_ * 2 + ((i) == 31)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                         \
  } while (0)

#include "../kd-via-fm-in-asr_amd/csrc/ffn.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

static float* dev_rand(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  srand(seed);
  for (auto& v : h) v = scale * ((rand() / (float)RAND_MAX) * 2.f - 1.f);
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

static void run(int64_t rows, int d, float p) {
  const int ff = 4 * d;
  float* x = dev_rand(rows * d, 1.f, 1);
  float* W1 = dev_rand((size_t)ff * d, 0.1f, 2);
  float* W2 = dev_rand((size_t)d * ff, 0.05f, 3);
  float* g = dev_rand(d, 0.f, 4);
  float *b, *b1, *b2, *out, *mean, *rstd;
  CK(hipMalloc(&b, d * 4));
  CK(hipMalloc(&b1, ff * 4));
  CK(hipMalloc(&b2, d * 4));
  CK(hipMemset(b, 0, d * 4));
  CK(hipMemset(b1, 0, ff * 4));
  CK(hipMemset(b2, 0, d * 4));
  CK(hipMalloc(&out, rows * d * 4));
  CK(hipMalloc(&mean, rows * 4));
  CK(hipMalloc(&rstd, rows * 4));
  uint16_t* img;
  CK(hipMalloc(&img, kdfm_ffn_img_elems(d, ff) * 2));
  if (kdfm_ffn_wprep(W1, W2, img, d, ff, 1, nullptr)) exit(2);
  uint64_t* seed;
  CK(hipMalloc(&seed, 8));
  CK(hipMemset(seed, 7, 8));
  const int64_t nblk = (rows + 63) / 64;
  unsigned long long *pb, *rt;
  CK(hipMalloc(&pb, nblk * 16 * 32 * 8));
  CK(hipMalloc(&rt, nblk * 16 * 2 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_pb), &pb, sizeof(pb)));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_rt), &rt, sizeof(rt)));
  auto launch = [&]() {
    if (kdfm_ffn_fwd(x, g, b, 1e-5f, img, b1, b2, out, mean, rstd, rows, d, ff, 0.5f, p, p, seed, 1, 2, nullptr,
                     nullptr, 0.f, nullptr, nullptr, nullptr, nullptr))
      exit(3);
  };
  for (int i = 0; i < 5; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipMemset(pb, 0, nblk * 16 * 32 * 8));
  CK(hipMemset(rt, 0, nblk * 16 * 2 * 8));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(nblk * 16 * 32), hr(nblk * 16 * 2);
  CK(hipMemcpy(h.data(), pb, h.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), rt, hr.size() * 8, hipMemcpyDeviceToHost));
  // per probe: average cycles since probe 0 over the waves that recorded it
  double sum[32] = {0}, cnt[32] = {0};
  double cyc = 0, rts = 0;
  int ncal = 0;
  unsigned long long t0min = ~0ull, tendmax = 0;
  for (int64_t w = 0; w < nblk * 16; ++w) {
    const unsigned long long* q = &h[w * 32];
    if (!q[0]) continue;
    t0min = q[0] < t0min ? q[0] : t0min;
    for (int i = 1; i < 32; ++i)
      if (q[i]) {
        sum[i] += (double)(q[i] - q[0]);
        cnt[i] += 1;
        tendmax = q[i] > tendmax ? q[i] : tendmax;
      }
    if (q[31] && hr[w * 2 + 1]) {
      cyc += (double)(q[31] - q[0]);
      rts += (double)(hr[w * 2 + 1] - hr[w * 2]);
      ++ncal;
    }
  }
  const double mhz = rts > 0 ? cyc / rts * 100.0 : 0.0;   // real-time clock: 100 MHz
  printf("ffn_fwd rows=%lld d=%d p=%.1f: %.1f us per launch (events, 20 launches); shader clock %.0f MHz; "
         "first-to-last wave span %.1f us\n",
         (long long)rows, d, p, 1e3 * ms / 20, mhz, mhz > 0 ? (tendmax - t0min) / mhz : 0.0);
  for (int i = 1; i < 32; ++i)
    if (cnt[i] > 0)
      printf("  probe %2d: %8.0f cycles (%6.2f us) after start, %6.0f waves\n", i, sum[i] / cnt[i],
             mhz > 0 ? sum[i] / cnt[i] / mhz : 0.0, cnt[i]);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 12832;
  run(rows, 88, 0.1f);
  run(rows, 176, 0.f);
  run(64, 88, 0.1f);
  run(64, 176, 0.f);
  return 0;
}
