// Library identity, error reporting and small reductions shared by all ops.
#include <cstring>
#include <string>

#include "common.h"

namespace kdfm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return KDFM_ELAUNCH;
  }
  return KDFM_OK;
}

namespace {
// out[n] (+)= scale * sum_{m<M} X[m*ld + n]  (bias gradients: N <= 2048, M up to ~2e5 rows).
// Each block streams a slab of rows in flat (coalesced) order, accumulates per column in LDS with
// LDS float atomics, then issues one global atomic per column.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, float* __restrict__ out,
                                                     int64_t M, int64_t N, int64_t ld, int64_t rows_per, float scale) {
  __shared__ float acc[2048];
  for (int64_t c = threadIdx.x; c < N; c += 256) acc[c] = 0.f;
  __syncthreads();
  const int64_t mb = (int64_t)blockIdx.x * rows_per;
  const int64_t me = (mb + rows_per < M) ? mb + rows_per : M;
  if (me > mb) {
    const int64_t cnt = (me - mb) * N;
    if (ld == N) {
      const float* base = X + mb * N;
      int64_t c = threadIdx.x % N;
      const int64_t step_c = 256 % N;
      float part = 0.f;
      for (int64_t i = threadIdx.x; i < cnt; i += 256) {
        // column of element i advances by 256 % N each iteration; flush when it wraps
        const float v = base[i];
        atomicAdd(&acc[c], v);
        c += step_c;
        if (c >= N) c -= N;
      }
      (void)part;
    } else {
      for (int64_t i = threadIdx.x; i < cnt; i += 256) {
        const int64_t r = i / N, c = i - r * N;
        atomicAdd(&acc[c], X[(mb + r) * ld + c]);
      }
    }
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < N; c += 256) atomicAdd(out + c, scale * acc[c]);
}

__global__ void zero_kernel(float* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = 0.f;
}
}  // namespace

}  // namespace kdfm

extern "C" {

const char* kdfm_version(void) { return "kdfm 0.1.0 (gfx950)"; }

const char* kdfm_last_error(void) { return kdfm::g_last_error.c_str(); }

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

int kdfm_colsum(const float* X, float* out, int64_t M, int64_t N, int64_t ld, float scale, int32_t accumulate,
                void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(X && out, "null pointer");
  KDFM_REQUIRE(M >= 0 && N >= 0 && ld >= N && N <= 2048, "bad shape (N <= 2048)");
  hipStream_t st = as_stream(stream);
  if (!accumulate) {
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, st, out, N);
    int rc = check_launch("kdfm_colsum(zero)");
    if (rc) return rc;
  }
  if (M == 0 || N == 0) return KDFM_OK;
  // ~16K elements per block, at most 1024 blocks
  int64_t rows_per = ceil_div(16384, N);
  if (ceil_div(M, rows_per) > 1024) rows_per = ceil_div(M, 1024);
  const int64_t gx = ceil_div(M, rows_per);
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)gx), dim3(256), 0, st, X, out, M, N, ld, rows_per, scale);
  return check_launch("kdfm_colsum");
}

}  // extern "C"
