// Library identity, error reporting and small reductions shared by all ops.
#include <cstring>
#include <string>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "common.h"

#include <vector>

namespace kdfm {

static thread_local std::string g_last_error;
static int g_deterministic = 0;
static thread_local int g_route = -1;

void set_error(const std::string& msg) { g_last_error = msg; }
bool deterministic() { return g_deterministic != 0; }
void set_route(int r) { g_route = r; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return KDFM_ELAUNCH;
  }
  return KDFM_OK;
}

namespace {
// out[n] (+)= scale * sum_{m<M} X[m*ld + n].  grid = (column groups of 64, row slabs); lane owns a
// column, the 4 waves stride the slab's rows with 4 independent accumulators each (latency hiding),
// LDS combine, one global atomic per column per block.
// out[n] += scale * sum_m X[m, n]; with out2, the columns n >= n1 go to out2[n - n1] instead (two
// adjacent partial blocks, e.g. a weight and a bias gradient, folded by one launch)
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, float* __restrict__ out,
                                                     float* __restrict__ out2, int64_t n1, int64_t M, int64_t N,
                                                     int64_t ld, int64_t rows_per, float scale) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + lane;
  const int64_t mb = (int64_t)blockIdx.y * rows_per;
  const int64_t me = (mb + rows_per < M) ? mb + rows_per : M;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (n < N) {
    int64_t m = mb + w;
    for (; m + 12 < me; m += 16) {
      s0 += X[m * ld + n];
      s1 += X[(m + 4) * ld + n];
      s2 += X[(m + 8) * ld + n];
      s3 += X[(m + 12) * ld + n];
    }
    for (; m < me; m += 4) s0 += X[m * ld + n];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && n < N)
    atomicAdd((out2 && n >= n1) ? out2 + (n - n1) : out + n,
              scale * (red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]));
}

__global__ void zero_kernel(float* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = 0.f;
}
}  // namespace

int launch_colsum(const float* X, float* out, int64_t M, int64_t N, int64_t ld, float scale, hipStream_t st) {
  return launch_colsum2(X, out, N, nullptr, M, N, ld, scale, st);
}

int launch_colsum2(const float* X, float* out, int64_t n1, float* out2, int64_t M, int64_t N, int64_t ld, float scale,
                   hipStream_t st) {
  if (M == 0 || N == 0) return KDFM_OK;
  const int64_t gx = ceil_div(N, 64);
  int64_t gy = ceil_div(M, 128);
  if (gy * gx > 2048) gy = (2048 + gx - 1) / gx;
  if (gy < 1 || deterministic()) gy = 1;  // one block per column group: a fixed summation order
  const int64_t rows_per = ceil_div(M, gy);
  gy = ceil_div(M, rows_per);
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st, X, out, out2, n1, M, N, ld,
                     rows_per, scale);
  return check_launch("colsum");
}

}  // namespace kdfm

extern "C" {

const char* kdfm_version(void) { return "kdfm 0.1.0 (gfx950)"; }

const char* kdfm_last_error(void) { return kdfm::g_last_error.c_str(); }

void kdfm_set_deterministic(int32_t on) { kdfm::g_deterministic = on ? 1 : 0; }

int32_t kdfm_get_deterministic(void) { return kdfm::g_deterministic; }

int32_t kdfm_gemm_last_route(void) { return kdfm::g_route; }

int32_t kdfm_range_push(const char* name) { return roctxRangePushA(name ? name : "kdfm"); }

int32_t kdfm_range_pop(void) { return roctxRangePop(); }

int kdfm_device_arch(char* buf, int64_t len) {
  KDFM_REQUIRE(buf && len > 0, "null buffer");
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    kdfm::set_error("kdfm_device_arch: no HIP device");
    return KDFM_ELAUNCH;
  }
  std::strncpy(buf, prop.gcnArchName, (size_t)len - 1);
  buf[len - 1] = 0;
  return KDFM_OK;
}

// stream-ordering and memset primitives of the step-plan replay (kdfm/plan.py): the recorded step's
// cross-stream edges and zero fills re-issued without going through torch
int kdfm_event_record(void* event, void* stream) {
  if (hipEventRecord(static_cast<hipEvent_t>(event), kdfm::as_stream(stream)) != hipSuccess) {
    kdfm::set_error("kdfm_event_record: hipEventRecord failed");
    return KDFM_ELAUNCH;
  }
  return KDFM_OK;
}

// cross-stream link events: hipEventDisableTiming plus the caller's release scope flags (the step's links pass
// hipEventReleaseToDevice / hipEventDisableSystemFence: a consumer on another stream of the same device needs the
// device-scope release every kernel boundary already has, not a system-scope fence)
int kdfm_event_create(void** event, uint32_t flags) {
  KDFM_REQUIRE(event, "null pointer");
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | flags) != hipSuccess) {
    kdfm::set_error("kdfm_event_create: hipEventCreateWithFlags failed");
    return KDFM_ELAUNCH;
  }
  *event = e;
  return KDFM_OK;
}

int kdfm_event_destroy(void* event) {
  if (event && hipEventDestroy(static_cast<hipEvent_t>(event)) != hipSuccess) {
    kdfm::set_error("kdfm_event_destroy: hipEventDestroy failed");
    return KDFM_ELAUNCH;
  }
  return KDFM_OK;
}

int kdfm_stream_wait_event(void* stream, void* event) {
  if (hipStreamWaitEvent(kdfm::as_stream(stream), static_cast<hipEvent_t>(event), 0) != hipSuccess) {
    kdfm::set_error("kdfm_stream_wait_event: hipStreamWaitEvent failed");
    return KDFM_ELAUNCH;
  }
  return KDFM_OK;
}

// A stream restricted to n_cus of the device's CUs (hipExtStreamCreateWithCUMask), spread uniformly over the
// CU index space (every (total / n_cus)-th CU, so whatever the index -> XCD mapping every XCD keeps its
// share): the weight-gradient stream runs its products beside the critical-path kernels without taking
// every CU's LDS and wave slots when its workgroups arrive first.  *out receives the hipStream_t.
int kdfm_stream_create_cu_mask(int32_t n_cus, void** out) {
  KDFM_REQUIRE(out && n_cus > 0, "bad arguments");
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    kdfm::set_error("kdfm_stream_create_cu_mask: no device");
    return KDFM_ELAUNCH;
  }
  const int total = prop.multiProcessorCount;
  KDFM_REQUIRE(n_cus <= total, "more CUs than the device has");
  std::vector<uint32_t> mask((size_t)(total + 31) / 32, 0u);
  for (int i = 0; i < n_cus; ++i) {
    const int cu = (int)(((int64_t)i * total) / n_cus);
    mask[(size_t)cu / 32] |= 1u << (cu % 32);
  }
  hipStream_t st = nullptr;
  if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    kdfm::set_error("kdfm_stream_create_cu_mask: hipExtStreamCreateWithCUMask failed");
    return KDFM_ELAUNCH;
  }
  *out = st;
  return KDFM_OK;
}

int kdfm_memset_async(void* ptr, int32_t value, int64_t bytes, void* stream) {
  KDFM_REQUIRE(ptr || bytes == 0, "null pointer");
  if (bytes == 0) return KDFM_OK;
  if (hipMemsetAsync(ptr, value, (size_t)bytes, kdfm::as_stream(stream)) != hipSuccess) {
    kdfm::set_error("kdfm_memset_async: hipMemsetAsync failed");
    return KDFM_ELAUNCH;
  }
  return KDFM_OK;
}

int kdfm_colsum(const float* X, float* out, int64_t M, int64_t N, int64_t ld, float scale, int32_t accumulate,
                void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(X && out, "null pointer");
  KDFM_REQUIRE(M >= 0 && N >= 0 && ld >= N, "bad shape");
  hipStream_t st = as_stream(stream);
  if (!accumulate) {
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, st, out, N);
    int rc = check_launch("kdfm_colsum(zero)");
    if (rc) return rc;
  }
  return launch_colsum(X, out, M, N, ld, scale, st);
}

}  // extern "C"
