// bf16 twins of the f32 parameter buffers (kdfm_gemm_desc.Bh): a plain cast for the [out][in]
// layout the forward products read, and an in-place-of-itself transpose of every 2-D weight for
// the data-gradient products (dX = dY W reads W^T rows).  Run once per step (the student's
// weights change every optimizer step; both casts are captured in the step graph).
#include "common.h"

namespace kdfm {
namespace {

__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                        int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 v = *reinterpret_cast<const float4*>(src + i);
    const uint32_t lo = pack_bf16x2(v.x, v.y);
    const uint32_t hi = pack_bf16x2(v.z, v.w);
    *reinterpret_cast<uint2*>(dst + i) = make_uint2(lo, hi);
  } else {
    for (int64_t j = i; j < n; ++j) dst[j] = f2bf(src[j]);
  }
}

// table rows: (offset, rows, cols, first_block); blocks of 256 elements of the OUTPUT (transposed)
// order so the 2-byte stores are contiguous; the f32 reads are strided by cols (L2-resident weights).
__global__ __launch_bounds__(256) void cast_bf16_t_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                          const int64_t* __restrict__ tab, int64_t ntab) {
  const int64_t blk = blockIdx.x;
  int64_t lo = 0, hi = ntab - 1;
  while (lo < hi) {  // last entry with first_block <= blk
    const int64_t mid = (lo + hi + 1) >> 1;
    if (tab[mid * 4 + 3] <= blk) lo = mid; else hi = mid - 1;
  }
  const int64_t off = tab[lo * 4 + 0], rows = tab[lo * 4 + 1], cols = tab[lo * 4 + 2], fb = tab[lo * 4 + 3];
  const int64_t e = (blk - fb) * 256 + threadIdx.x;  // index in the transposed image: e = c*rows + r
  if (e >= rows * cols) return;
  const int64_t c = e / rows, r = e - c * rows;
  dst[off + e] = f2bf(src[off + r * cols + c]);
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_cast_bf16(const float* src, uint16_t* dst, int64_t n, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(src && dst && n >= 0, "bad arguments");
  KDFM_REQUIRE((((uintptr_t)src) & 15) == 0 && (((uintptr_t)dst) & 7) == 0, "src 16-B / dst 8-B aligned");
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)ceil_div(ceil_div(n, 4), 256)), dim3(256), 0, as_stream(stream),
                     src, dst, n);
  return check_launch("kdfm_cast_bf16");
}

int kdfm_cast_bf16_t(const float* src, uint16_t* dst, const int64_t* table, int64_t ntab, int64_t nblocks,
                     void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(src && dst && table && ntab > 0 && nblocks > 0, "bad arguments");
  hipLaunchKernelGGL(cast_bf16_t_kernel, dim3((unsigned)nblocks), dim3(256), 0, as_stream(stream), src, dst, table,
                     ntab);
  return check_launch("kdfm_cast_bf16_t");
}

}  // extern "C"
