// kdfm — shared device/host helpers for the gfx950 kernels behind libkdfm.so.
//
// Storage convention: every activation/gradient tensor is fp32 in HBM, channels-last
// (rows = utterance-major frames, columns = features). MFMA operands are converted to bf16
// (throughput mode) or fed as exact f32 (parity mode) at LDS-staging time.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/kdfm.h"

namespace kdfm {

// ---- error handling -------------------------------------------------------------------------
void set_error(const std::string& msg);
int check_launch(const char* what);
// Deterministic-reduction mode (kdfm_set_deterministic): every reduction that feeds an activation
// or a gradient runs in a fixed order (no split-K / cross-block float atomics), so two runs on the
// same inputs give bitwise-identical results.  Read on the host when a launch is configured.
bool deterministic();
// Kernel family the most recent kdfm_gemm call on this thread launched (kdfm_gemm_last_route):
// 0 generic 64x64 tile, 1 weight-stationary skinny, 2 row-streaming forward, 3 wide-tile weight
// gradient (+ fold), 4 generic with ordered split-K fold, 5 LDS-slab k=3 conv, 6 row-parallel
// weight gradient (+ ordered fold).
enum { ROUTE_GENERIC = 0, ROUTE_SKINNY = 1, ROUTE_RS_FWD = 2, ROUTE_RS_WGRAD = 3, ROUTE_SPLIT_FOLD = 4,
       ROUTE_SLAB_CONV = 5, ROUTE_WGRAD_ROWS = 6, ROUTE_BIG = 7 };
void set_route(int r);

#define KDFM_REQUIRE(cond, msg)                                  \
  do {                                                           \
    if (!(cond)) {                                               \
      ::kdfm::set_error(std::string(__func__) + ": " + (msg));   \
      return KDFM_EINVAL;                                        \
    }                                                            \
  } while (0)

// ---- small math -------------------------------------------------------------------------------
__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ uint16_t f2bf(float f) {
  // round-to-nearest-even; NaN handled by the plain cast path in hipcc (v_cvt_pk_bf16_f32)
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

// two floats -> packed bf16 pair (lo = a, hi = b), round-to-nearest-even: ONE v_cvt_pk_bf16_f32 (two
// scalar f2bf calls cost a convert each plus a shift and an or)
typedef __bf16 kdfm_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float kdfm_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const kdfm_f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, kdfm_bf16x2_t));
}

// 8 floats -> 8 packed bf16 (4 converts), as the 16-byte MFMA operand vector type V
template <typename V>
__device__ __forceinline__ V pack_bf16x8(const float* v) {
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t w = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
  return __builtin_bit_cast(V, w);
}

// v_rcp_f32 (1 ulp) instead of the IEEE division sequence (div_scale / div_fmas / div_fixup, ~10 VALU
// ops per element): the SiLU / GLU epilogues of the fused LN-block kernels were VALU-bound on it
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float siluf_(float x) { return x * sigmoidf_(x); }
__device__ __forceinline__ float dsiluf_(float x) {
  float s = sigmoidf_(x);
  return s * (1.f + x * (1.f - s));
}

// ---- counter-based RNG (dropout masks, SpecAugment draws, NoiseAdapter eps) -----------------
// splitmix64-style finaliser over (seed, stream, index): the same triple always yields the same
// bits, so backward kernels regenerate the forward's dropout mask instead of storing it.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// (seed, stream) -> per-stream key (uniform per launch: the compiler keeps it scalar), then ONE
// splitmix64 finaliser per element at counter position idx of that key's sequence
__host__ __device__ __forceinline__ uint64_t rng_key(uint64_t seed, uint64_t stream) {
  return mix64(seed ^ mix64(stream * 0x2545F4914F6CDD1Dull));
}
__device__ __forceinline__ uint64_t rng_bits_k(uint64_t key, uint64_t idx) {
  return mix64(key + idx * 0x9E3779B97F4A7C15ull);
}
__device__ __forceinline__ uint64_t rng_bits(uint64_t seed, uint64_t stream, uint64_t idx) {
  return rng_bits_k(rng_key(seed, stream), idx);
}
__device__ __forceinline__ float rng_uniform(uint64_t seed, uint64_t stream, uint64_t idx) {
  return (float)(rng_bits(seed, stream, idx) >> 40) * (1.0f / 16777216.0f);  // [0,1)
}
__device__ __forceinline__ float rng_normal(uint64_t seed, uint64_t stream, uint64_t idx) {
  uint64_t b = rng_bits(seed, stream, idx);
  float u1 = ((float)(b >> 40) + 1.0f) * (1.0f / 16777217.0f);  // (0,1]
  float u2 = (float)((b >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}
// Dropout decisions are the hottest RNG use (every FFN / attention / residual element of a training
// step).  One 32-bit keyed hash per PAIR of elements (2 * pair, 2 * pair + 1): the pair index times an
// odd per-stream multiplier plus a per-stream offset, then one lowbias32 round (3 v_mul_lo_u32 per pair
// in all, vs 12 per element for a 64-bit splitmix finaliser); each element of the pair tests 16 of the
// 32 bits.  keep iff u16 >= ceil(p * 65536): P(drop) = ceil(p * 2^16) / 2^16 (p = 0.1 -> 0.1000061).
__host__ __device__ __forceinline__ uint32_t drop_pair_bits(uint64_t key, uint64_t pair) {
  uint32_t x = (uint32_t)pair * ((uint32_t)(key >> 32) | 1u) + (uint32_t)key;
  x ^= (uint32_t)(pair >> 32);
  x ^= x >> 16;
  x *= 0x21f0aaadu;
  x ^= x >> 15;
  x *= 0x735a2d97u;
  x ^= x >> 15;
  return x;
}
__device__ __forceinline__ uint32_t drop_threshold(float p) { return (uint32_t)ceilf(p * 65536.f); }
// dropout keep test on a precomputed key (rng_key(seed, stream)) for flat element index idx
__device__ __forceinline__ bool dropout_keep_k(uint64_t key, uint64_t idx, float p) {
  const uint32_t h = drop_pair_bits(key, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xffffu)) >= drop_threshold(p);
}
// the two decisions of elements idx_even and idx_even + 1 (idx_even even) from one hash
__device__ __forceinline__ void dropout_keep2_k(uint64_t key, uint64_t idx_even, float p, bool& k0, bool& k1) {
  const uint32_t h = drop_pair_bits(key, idx_even >> 1);
  const uint32_t t = drop_threshold(p);
  k0 = (h & 0xffffu) >= t;
  k1 = (h >> 16) >= t;
}
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t stream, uint64_t idx, float p) {
  return dropout_keep_k(rng_key(seed, stream), idx, p);
}
// Attention-probability dropout of element (row, key j) of a T x T map, row = (b H + h) T + i: one hash per
// (row, key pair j >> 1) -- pair index row * ceil(T / 2) + (j >> 1), so a pair never straddles two rows and
// keys 2m, 2m + 1 (neighbouring lanes of an MFMA C tile) share it -- and 16 bits per key (j & 1 picks them).
// Every attention kernel (fused forwards, bwd2, the unfused softmax) draws its mask through this.
__host__ __device__ __forceinline__ uint64_t attn_drop_rowpairs(int64_t row, int64_t T) {
  return (uint64_t)row * (uint64_t)((T + 1) >> 1);
}
__device__ __forceinline__ bool attn_drop_keep(uint64_t key, uint64_t rowpairs, int64_t j, float p) {
  const uint32_t h = drop_pair_bits(key, rowpairs + (uint64_t)(j >> 1));
  return ((j & 1) ? (h >> 16) : (h & 0xffffu)) >= drop_threshold(p);
}
__device__ __forceinline__ uint64_t load_seed(const uint64_t* seed_ptr) { return seed_ptr ? *seed_ptr : 0ull; }

// ---- wave64 reductions --------------------------------------------------------------------------
// XCD-aware block order for 1-D grids.  The dispatcher deals consecutive workgroups round-robin
// to the 8 XCDs, each with its own L2: neighbouring blocks that share input lines (gathers such as
// col2im / im2col, whose taps overlap) would fetch the same lines once per XCD.  This bijection
// gives XCD x a CONTIGUOUS range of logical blocks instead, so the overlap is served by one L2.
constexpr int kNumXcd = 8;
__device__ __forceinline__ int64_t xcd_block() {
  const int64_t b = blockIdx.x, n = gridDim.x;
  const int64_t x = b % kNumXcd, local = b / kNumXcd;
  const int64_t per = n / kNumXcd, rem = n % kNumXcd;
  return x < rem ? x * (per + 1) + local : rem * (per + 1) + (x - rem) * per + local;
}
// The same bijection over a 3-D grid (dispatched x fastest, then y, then z): returns the logical
// block (bx, by, bz).  Attention grids put the blocks of one (utterance, head) along x, so they
// land on one XCD and share its L2 for K / V / positions instead of fetching them once per XCD.
struct Blk3 { int64_t x, y, z; };
__device__ __forceinline__ int64_t xcd_linear() {
  const int64_t nx = gridDim.x, ny = gridDim.y;
  const int64_t b = blockIdx.x + nx * (blockIdx.y + ny * (int64_t)blockIdx.z);
  const int64_t n = nx * ny * (int64_t)gridDim.z;
  const int64_t x = b % kNumXcd, local = b / kNumXcd;
  const int64_t per = n / kNumXcd, rem = n % kNumXcd;
  return x < rem ? x * (per + 1) + local : rem * (per + 1) + (x - rem) * per + local;
}
__device__ __forceinline__ Blk3 xcd_block3() {
  const int64_t nx = gridDim.x, ny = gridDim.y, l = xcd_linear();
  return Blk3{l % nx, (l / nx) % ny, l / (nx * ny)};
}
// y-fastest variant for GEMM grids (x = row tiles, y = column tiles): the column tiles of one row
// block share its A rows, so they go to the same XCD.
__device__ __forceinline__ Blk3 xcd_block3_yfast() {
  const int64_t nx = gridDim.x, ny = gridDim.y, l = xcd_linear();
  const int64_t r = l % (nx * ny);
  return Blk3{r / ny, r % ny, l / (nx * ny)};
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum for blockDim.x multiple of 64 (<= 1024); `red` must hold >= 16 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// out[n] += scale * sum_m X[m*ld + n]  (n < N); defined in runtime.hip.  Used to fold per-block
// column partials written by reduction-heavy backward kernels (deterministic, no hot atomics).
int launch_colsum(const float* X, float* out, int64_t M, int64_t N, int64_t ld, float scale, hipStream_t st);
int launch_colsum2(const float* X, float* out, int64_t n1, float* out2, int64_t M, int64_t N, int64_t ld, float scale,
                   hipStream_t st);

}  // namespace kdfm
