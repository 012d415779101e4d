// Operand lane-map probe of the block-scaled fp8 MFMA v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, unit
// e8m0 scales): every lane loads its 32 raw operand bytes of A and B from host-prepared arrays, one MFMA, and
// writes its 4 accumulator values (C/D map: col = lane & 15, row = 4 (lane >> 4) + r, dtype-independent on gfx950).
// tools/fp8_probe.py prepares the bytes under a hypothesised lane map and checks C against an exact reference.
// Build: hipcc -O2 -shared -fPIC --offload-arch=gfx950 tools/fp8_probe.hip -o tools/fp8_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void probe_kernel(const int* a, const int* b, float* c, int sa, int sb, const int* lsa, const int* lsb) {
  const int l = threadIdx.x;
  if (lsa) {   // per-lane e8m0 scales (MX block scaling: one per lane = per 32 k-elements of one row / column)
    sa = lsa[l];
    sb = lsb[l];
  }
  v8i av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[l * 8 + i];
    bv[i] = b[l * 8 + i];
  }
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) c[l * 4 + r] = acc[r];
}

extern "C" int fp8_probe(const int* a, const int* b, float* c, int sa, int sb, const int* lsa, const int* lsb) {
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, 0, a, b, c, sa, sb, lsa, lsb);
  return (int)hipDeviceSynchronize();
}

// scale-slot probe: block t of the grid runs one MFMA on its own operands (a, b: [nb][64 lanes][8 words]) with its
// own per-lane scales (lsa, lsb: [nb][64]) and writes its accumulators to c[t][64][4]
__global__ void probe_batch_kernel(const int* a, const int* b, float* c, const int* lsa, const int* lsb) {
  const int l = threadIdx.x, t = blockIdx.x;
  v8i av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[(t * 64 + l) * 8 + i];
    bv[i] = b[(t * 64 + l) * 8 + i];
  }
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, lsa[t * 64 + l], 0, lsb[t * 64 + l]);
  for (int r = 0; r < 4; ++r) c[(t * 64 + l) * 4 + r] = acc[r];
}

// the same with the accumulator read from c (so the destination registers are not the scale registers) and idle
// cycles between the scale loads and the MFMA
__global__ void probe_batch2_kernel(const int* a, const int* b, float* c, const int* lsa, const int* lsb) {
  const int l = threadIdx.x, t = blockIdx.x;
  v8i av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[(t * 64 + l) * 8 + i];
    bv[i] = b[(t * 64 + l) * 8 + i];
  }
  int sa = lsa[t * 64 + l], sb = lsb[t * 64 + l];
  v4f acc;
  for (int r = 0; r < 4; ++r) acc[r] = c[(t * 64 + l) * 4 + r];
  asm volatile("s_waitcnt vmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7" : "+v"(sa), "+v"(sb), "+v"(acc));
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) c[(t * 64 + l) * 4 + r] = acc[r];
}

// batch2 with the scale registers overwritten right after the MFMA issues (a write-after-read on the scale operands)
__global__ void probe_batch3_kernel(const int* a, const int* b, float* c, const int* lsa, const int* lsb) {
  const int l = threadIdx.x, t = blockIdx.x;
  v8i av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[(t * 64 + l) * 8 + i];
    bv[i] = b[(t * 64 + l) * 8 + i];
  }
  int sa = lsa[t * 64 + l], sb = lsb[t * 64 + l];
  v4f acc;
  for (int r = 0; r < 4; ++r) acc[r] = c[(t * 64 + l) * 4 + r];
  asm volatile("s_waitcnt vmcnt(0)\n s_nop 7" : "+v"(sa), "+v"(sb), "+v"(acc));
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, sb);
  asm volatile("v_mov_b32 %0, 0\n v_mov_b32 %1, 0" : "+v"(sa), "+v"(sb));
  for (int r = 0; r < 4; ++r) c[(t * 64 + l) * 4 + r] = acc[r] + 0.f * (float)(sa + sb);
}

extern "C" int fp8_probe_batch3(const int* a, const int* b, float* c, const int* lsa, const int* lsb, int nb) {
  hipLaunchKernelGGL(probe_batch3_kernel, dim3(nb), dim3(64), 0, 0, a, b, c, lsa, lsb);
  return (int)hipDeviceSynchronize();
}

extern "C" int fp8_probe_batch(const int* a, const int* b, float* c, const int* lsa, const int* lsb, int nb) {
  if (nb < 0) {
    hipLaunchKernelGGL(probe_batch2_kernel, dim3(-nb), dim3(64), 0, 0, a, b, c, lsa, lsb);
    return (int)hipDeviceSynchronize();
  }
  hipLaunchKernelGGL(probe_batch_kernel, dim3(nb), dim3(64), 0, 0, a, b, c, lsa, lsb);
  return (int)hipDeviceSynchronize();
}

// f32 -> fp8 conversion check: v_cvt_pk_fp8_f32 (the builtin biggemm.hip's quantizer uses) on n inputs, byte out
__global__ void cvt_kernel(const float* x, unsigned char* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const int w = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
  y[2 * i] = (unsigned char)(w & 0xFF);
  y[2 * i + 1] = (unsigned char)((w >> 8) & 0xFF);
}

extern "C" int fp8_cvt(const float* x, unsigned char* y, int n) {
  hipLaunchKernelGGL(cvt_kernel, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, x, y, n);
  return (int)hipDeviceSynchronize();
}
