// Batched GEMM with fused epilogues on gfx950 MFMA.
//
// One kernel template covers every matmul-shaped op of the ver5 step (see include/kdfm.h,
// kdfm_gemm).  Block = 256 threads (4 waves), block tile 64x64, K-step 32.  Each wave owns a
// 32x32 quadrant computed as 2x2 MFMA tiles of 16x16:
//   BF16: v_mfma_f32_16x16x32_bf16, LDS image [m][k] (k contiguous, 16-B fragment reads)
//   F32 : v_mfma_f32_16x16x4_f32 (exact f32), LDS image [k][m] (conflict-free b32 reads)
// Global->register prefetch of tile t+1 overlaps the MFMAs of tile t (T14 split).
#include "gemm_common.h"

namespace kdfm {
namespace {

constexpr int BM = 64, BN = 64, BK = 32, NT = 256;
constexpr int KSUB_BF = 2;                 // bf16: two 32-wide k halves per iteration (BK 64)
constexpr int LDK_BF = BK * KSUB_BF + 8;   // bf16 image row stride (elements)
constexpr int LDX_F32 = BM + 16; // f32 image row stride (elements) -> lanes 16..31 on banks +16

using P = GemmP;

// Operand element fetch for the "row operand" view: X(r, q) where r is the row-like index
// (m for A, n for B) and q the contraction index k.  Returns 0 outside bounds.
template <int MODE>
__device__ __forceinline__ float fetch(const float* base, int64_t r, int64_t q, int64_t R, int64_t Q,
                                       int64_t sr, int64_t sq, const P& p) {
  if (r >= R || q >= Q) return 0.f;
  if constexpr (MODE == KDFM_LD_CONV) {
    // A: r = m (frame row), q = k = tap*C + c   ->  x[m + tap - pad][c]
    const int64_t tap = q / p.conv_c, c = q - tap * p.conv_c;
    const int64_t t = r % p.conv_t;
    const int64_t tt = t + tap - p.pad;
    if (tt < 0 || tt >= p.conv_t) return 0.f;
    return base[(r + tap - p.pad) * sr + c * sq];
  } else {
    return base[r * sr + q * sq];
  }
}

// B operand in CONV mode: B(k, n) with k the frame row and n = tap*C + c -> x[k + tap - pad][c]
__device__ __forceinline__ float fetch_bconv(const float* base, int64_t k, int64_t n, int64_t K, int64_t N,
                                             int64_t sk, int64_t sn, const P& p) {
  if (k >= K || n >= N) return 0.f;
  const int64_t tap = n / p.conv_c, c = n - tap * p.conv_c;
  const int64_t t = k % p.conv_t;
  const int64_t tt = t + tap - p.pad;
  if (tt < 0 || tt >= p.conv_t) return 0.f;
  return base[(k + tap - p.pad) * sk + c * sn];
}

// Each thread stages 8 elements of a 64x32 (rows x k) operand tile.
//  KC/CONV mode: thread -> (row = t>>2, k0 = (t&3)*8), 8 consecutive k
//  XC mode     : thread -> (k = t>>3, r0 = (t&7)*8), 8 consecutive rows
template <int MODE>
__device__ __forceinline__ void load_tile_A(float (&v)[8], const float* base, int64_t r0, int64_t k0,
                                            int64_t R, int64_t Q, int64_t sr, int64_t sq, const P& p) {
  const int t = threadIdx.x;
  if constexpr (MODE == KDFM_LD_XC) {
    const int64_t k = k0 + (t >> 3), r = r0 + (t & 7) * 8;
    if (sr == 1 && k < Q && r + 7 < R && ((((uintptr_t)(base + r + k * sq)) & 15) == 0)) {
      const float4* q4 = reinterpret_cast<const float4*>(base + r + k * sq);
      float4 a = q4[0], b = q4[1];
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fetch<KDFM_LD_KC>(base, r + i, k, R, Q, sr, sq, p);
    }
  } else {
    const int64_t r = r0 + (t >> 2), k = k0 + (t & 3) * 8;
    if constexpr (MODE == KDFM_LD_CONV) {
      // 8 consecutive k stay inside one tap when conv_c % 8 == 0: one validity test, 2x dwordx4
      if (sq == 1 && (p.conv_c & 7) == 0 && r < R && k + 7 < Q) {
        const int64_t tap = k / p.conv_c, c = k - tap * p.conv_c;
        const int64_t tt = (r % p.conv_t) + tap - p.pad;
        if (tt < 0 || tt >= p.conv_t) {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = 0.f;
          return;
        }
        const float* src = base + (r + tap - p.pad) * sr + c;
        if ((((uintptr_t)src) & 15) == 0) {
          const float4* q4 = reinterpret_cast<const float4*>(src);
          float4 a = q4[0], b = q4[1];
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
          return;
        }
      }
    }
    if (MODE == KDFM_LD_KC && sq == 1 && r < R && k + 7 < Q &&
        ((((uintptr_t)(base + r * sr + k)) & 15) == 0)) {
      const float4* q4 = reinterpret_cast<const float4*>(base + r * sr + k);
      float4 a = q4[0], b = q4[1];
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fetch<MODE>(base, r, k + i, R, Q, sr, sq, p);
    }
  }
}

// B operand tile (n rows x k) staging.  KC: B(k,n) contiguous along k (W[n][k]);
// XC: contiguous along n; CONV: k is a frame row, n = tap*C + c.
template <int MODE>
__device__ __forceinline__ void load_tile_B_mem(float (&v)[8], const float* base, int64_t n0, int64_t k0,
                                                int64_t N, int64_t K, int64_t sBk, int64_t sBn, const P& p) {
  const int t = threadIdx.x;
  if constexpr (MODE == KDFM_LD_KC) {
    load_tile_A<KDFM_LD_KC>(v, base, n0, k0, N, K, sBn, sBk, p);
  } else if constexpr (MODE == KDFM_LD_XC) {
    load_tile_A<KDFM_LD_XC>(v, base, n0, k0, N, K, sBn, sBk, p);
  } else {
    const int64_t k = k0 + (t >> 3), n = n0 + (t & 7) * 8;
    if (sBn == 1 && (p.conv_c & 7) == 0 && k < K && n + 7 < N) {
      const int64_t tap = n / p.conv_c, c = n - tap * p.conv_c;
      const int64_t tt = (k % p.conv_t) + tap - p.pad;
      if (tt < 0 || tt >= p.conv_t) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.f;
        return;
      }
      const float* src = base + (k + tap - p.pad) * sBk + c;
      if ((((uintptr_t)src) & 15) == 0) {
        const float4* q4 = reinterpret_cast<const float4*>(src);
        float4 a = q4[0], b = q4[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fetch_bconv(base, k, n + i, K, N, sBk, sBn, p);
  }
}

// B staging with the optional implicit ones column at n == ones_col (memory holds ones_col columns)
template <int MODE>
__device__ __forceinline__ void load_tile_B(float (&v)[8], const float* base, int64_t n0, int64_t k0,
                                            int64_t N, int64_t K, int64_t sBk, int64_t sBn, const P& p) {
  if (p.ones_col < 0) {
    load_tile_B_mem<MODE>(v, base, n0, k0, N, K, sBk, sBn, p);
    return;
  }
  load_tile_B_mem<MODE>(v, base, n0, k0, p.ones_col, K, sBk, sBn, p);
  const int t = threadIdx.x;
  if constexpr (MODE == KDFM_LD_KC) {
    const int64_t n = n0 + (t >> 2), k = k0 + (t & 3) * 8;
    if (n == p.ones_col)
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (k + i < K) ? 1.f : 0.f;
  } else {
    const int64_t k = k0 + (t >> 3), n = n0 + (t & 7) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (n + i == p.ones_col) v[i] = (k < K) ? 1.f : 0.f;
  }
}

// Write a staged 8-vector into the LDS image.  `kmajor_thread` = thread held 8 consecutive k.
template <bool BF16, bool KRUN>
__device__ __forceinline__ void store_lds(void* lds, const float (&v)[8], int khalf = 0) {
  const int t = threadIdx.x;
  if constexpr (BF16) {
    uint16_t* s = reinterpret_cast<uint16_t*>(lds) + khalf * BK;  // [64][LDK_BF], k half khalf
    if constexpr (KRUN) {
      const int r = t >> 2, k = (t & 3) * 8;
      *reinterpret_cast<bf16x8*>(s + r * LDK_BF + k) = pack_bf16x8<bf16x8>(v);
    } else {
      const int k = t >> 3, r = (t & 7) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) s[(r + i) * LDK_BF + k] = f2bf(v[i]);
    }
  } else {
    float* s = reinterpret_cast<float*>(lds);  // [32][LDX_F32]
    if constexpr (KRUN) {
      const int r = t >> 2, k = (t & 3) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) s[(k + i) * LDX_F32 + r] = v[i];
    } else {
      const int k = t >> 3, r = (t & 7) * 8;
      float4* d = reinterpret_cast<float4*>(s + k * LDX_F32 + r);
      d[0] = make_float4(v[0], v[1], v[2], v[3]);
      d[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

template <bool BF16, int AM, int BMODE, int EMODE = SKC_EPI_GENERIC>
__global__ __launch_bounds__(NT) void gemm_kernel(P p) {
  constexpr int LDS_ELEMS = BF16 ? (64 * LDK_BF / 2) : (BK * LDX_F32);  // in floats
  constexpr int KSUB = BF16 ? KSUB_BF : 1;   // 32-wide k halves per iteration
  constexpr int BKI = BK * KSUB;             // k per iteration (one barrier pair)
  __shared__ __attribute__((aligned(16))) float smem[2 * LDS_ELEMS];
  float* As = smem;
  float* Bs = smem + LDS_ELEMS;

  const Blk3 blk = xcd_block3_yfast();
  const int64_t z = blk.z;
  const int64_t split = z % p.splitk;
  const int64_t bz = z / p.splitk;
  const int64_t b1 = bz / p.batch2, b2 = bz % p.batch2;
  const float* A = p.A + b1 * p.bA1 + b2 * p.bA2;
  const float* B = p.B + b1 * p.bB1 + b2 * p.bB2;
  const int64_t cOff = b1 * p.bC1 + b2 * p.bC2;

  const int64_t m0 = blk.x * BM;
  const int64_t n0 = blk.y * BN;
  const int64_t kchunk = ceil_div(ceil_div(p.K, p.splitk), BKI) * BKI;
  const int64_t kbeg = split * kchunk;
  const int64_t kend = (kbeg + kchunk < p.K) ? (kbeg + kchunk) : p.K;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool A_KRUN = (AM != KDFM_LD_XC);
  constexpr bool B_KRUN = (BMODE == KDFM_LD_KC);

  float va[KSUB][8], vb[KSUB][8];
  auto load_it = [&](int64_t k0) {
#pragma unroll
    for (int hh = 0; hh < KSUB; ++hh) {
      load_tile_A<AM>(va[hh], A, m0, k0 + hh * BK, p.M, kend, p.sAm, p.sAk, p);
      load_tile_B<BMODE>(vb[hh], B, n0, k0 + hh * BK, p.N, kend, p.sBk, p.sBn, p);
    }
  };
  if (kbeg < kend) load_it(kbeg);
  for (int64_t k0 = kbeg; k0 < kend; k0 += BKI) {
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < KSUB; ++hh) {
      store_lds<BF16, A_KRUN>(As, va[hh], hh);
      store_lds<BF16, B_KRUN>(Bs, vb[hh], hh);
    }
    __syncthreads();
    if (k0 + BKI < kend) load_it(k0 + BKI);  // prefetch next tile into registers while the MFMAs run
    if constexpr (BF16) {
      const uint16_t* as = reinterpret_cast<const uint16_t*>(As);
      const uint16_t* bs = reinterpret_cast<const uint16_t*>(Bs);
#pragma unroll
      for (int hh = 0; hh < KSUB; ++hh) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(as + (wr * 32 + i * 16 + (lane & 15)) * LDK_BF + hh * BK +
                                                   8 * (lane >> 4));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(bs + (wc * 32 + j * 16 + (lane & 15)) * LDK_BF + hh * BK +
                                                    8 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        const int kr = kk + (lane >> 4);
        float a0 = As[kr * LDX_F32 + wr * 32 + (lane & 15)];
        float a1 = As[kr * LDX_F32 + wr * 32 + 16 + (lane & 15)];
        float b0 = Bs[kr * LDX_F32 + wc * 32 + (lane & 15)];
        float b1v = Bs[kr * LDX_F32 + wc * 32 + 16 + (lane & 15)];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1v, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1v, acc[1][1], 0, 0, 0);
      }
    }
  }

  // ---- epilogue ----
  const int epi = p.epi;
  uint64_t seed = 0;
  if (epi & KDFM_EPI_DROPOUT) seed = load_seed(p.seed);
  const float keep_scale = (epi & KDFM_EPI_DROPOUT) ? 1.f / (1.f - p.dropout_p) : 1.f;
  float mse_part = 0.f;
  bool single;
  const float* side = epi_side_src(p, single);
  if (!(epi & KDFM_EPI_ATOMIC) && single) {
    // two-phase: every side operand / bias / row-mask load first, then compute and store
    float sv[2][2][4], bnv[2][2];
    bool rok[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        rok[i][r] = m < p.M && epi_row_ok(p, m < p.M ? m : 0);
      }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wc * 32 + j * 16 + (lane & 15);
      bnv[j][0] = ((epi & KDFM_EPI_BIAS) && n < p.N) ? p.bias[n] : 0.f;
    }
    if (side) {
      const float* sb = side + cOff;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
            const int64_t n = n0 + wc * 32 + j * 16 + (lane & 15);
            sv[i][j][r] = (m < p.M && n < p.N) ? sb[m * p.sCm + n * p.sCn] : 0.f;
          }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
          const int64_t n = n0 + wc * 32 + j * 16 + (lane & 15);
          if (m >= p.M || n >= p.N) continue;
          const int64_t off = cOff + m * p.sCm + n * p.sCn;
          float pre = 0.f;
          const float v = skc_epi<EMODE>(p, m, n, p.alpha * acc[i][j][r], bnv[j][0], side ? sv[i][j][r] : 0.f,
                                         rok[i][r], seed, keep_scale, mse_part, pre, bz);
          if (epi & KDFM_EPI_STORE_PRE) p.Cpre[off] = pre;
          p.C[off] = v;
        }
  } else {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int64_t n = n0 + wc * 32 + j * 16 + (lane & 15);
        if (m >= p.M || n >= p.N) continue;
        const int64_t off = cOff + m * p.sCm + n * p.sCn;
        float v = p.alpha * acc[i][j][r];
        if (epi & KDFM_EPI_ATOMIC) {
          if (p.partial) {  // deterministic split-K: raw partial, folded in split order afterwards
            p.ws[(split * p.M + m) * p.N + n] = acc[i][j][r];
            continue;
          }
          if (n == p.ones_col)
            atomicAdd(p.ones_out + m, v);
          else
            atomicAdd(p.C + off, v);
          continue;
        }
        epilogue_store(p, bz, m, n, off, v, seed, keep_scale, mse_part);
      }
  }
  if (epi & KDFM_EPI_MSE) {
    mse_part = wave_sum(mse_part);
    if (lane == 0) atomicAdd(p.loss_acc, mse_part * p.loss_scale);
  }
}

template <bool BF16>
int launch(const P& p, int amode, int bmode, dim3 grid, hipStream_t st) {
  if constexpr (BF16) {
    // compile-time epilogues (gemm_common.h) for the bf16 row-operand products of the layers
    static const int fast = [] {
      const char* e = getenv("KDFM_SKC_FAST_EPI");
      return e ? atoi(e) : 1;
    }();
    const int em = fast ? skc_epi_mode(p.epi) : SKC_EPI_GENERIC;
    if (em != SKC_EPI_GENERIC && amode == KDFM_LD_KC && (bmode == KDFM_LD_KC || bmode == KDFM_LD_XC)) {
#define KDFM_GEMM_FAST(BMv, EMv)                                                           \
  if (bmode == BMv && em == EMv) {                                                         \
    hipLaunchKernelGGL((gemm_kernel<true, KDFM_LD_KC, BMv, EMv>), grid, dim3(NT), 0, st, p); \
    return check_launch("kdfm_gemm");                                                      \
  }
      KDFM_GEMM_FAST(KDFM_LD_KC, SKC_EPI_NONE)
      KDFM_GEMM_FAST(KDFM_LD_KC, SKC_EPI_RELU)
      KDFM_GEMM_FAST(KDFM_LD_KC, SKC_EPI_RESID)
      KDFM_GEMM_FAST(KDFM_LD_KC, SKC_EPI_DRELU)
      KDFM_GEMM_FAST(KDFM_LD_XC, SKC_EPI_NONE)
      KDFM_GEMM_FAST(KDFM_LD_XC, SKC_EPI_RELU)
      KDFM_GEMM_FAST(KDFM_LD_XC, SKC_EPI_RESID)
      KDFM_GEMM_FAST(KDFM_LD_XC, SKC_EPI_DRELU)
      KDFM_GEMM_FAST(KDFM_LD_KC, SKC_EPI_SILU_DROP)
      KDFM_GEMM_FAST(KDFM_LD_KC, SKC_EPI_DROP_RESID)
      KDFM_GEMM_FAST(KDFM_LD_XC, SKC_EPI_SILU_DROP)
      KDFM_GEMM_FAST(KDFM_LD_XC, SKC_EPI_DROP_RESID)
#undef KDFM_GEMM_FAST
    }
  }
#define KDFM_GEMM_CASE(AMv, BMv)                                                    \
  if (amode == AMv && bmode == BMv) {                                               \
    hipLaunchKernelGGL((gemm_kernel<BF16, AMv, BMv>), grid, dim3(NT), 0, st, p);    \
    return check_launch("kdfm_gemm");                                               \
  }
  KDFM_GEMM_CASE(KDFM_LD_KC, KDFM_LD_KC)
  KDFM_GEMM_CASE(KDFM_LD_KC, KDFM_LD_XC)
  KDFM_GEMM_CASE(KDFM_LD_KC, KDFM_LD_CONV)
  KDFM_GEMM_CASE(KDFM_LD_XC, KDFM_LD_KC)
  KDFM_GEMM_CASE(KDFM_LD_XC, KDFM_LD_XC)
  KDFM_GEMM_CASE(KDFM_LD_XC, KDFM_LD_CONV)
  KDFM_GEMM_CASE(KDFM_LD_CONV, KDFM_LD_KC)
  KDFM_GEMM_CASE(KDFM_LD_CONV, KDFM_LD_XC)
#undef KDFM_GEMM_CASE
  set_error("kdfm_gemm: unsupported operand mode combination");
  return KDFM_EUNSUPPORTED;
}

}  // namespace
}  // namespace kdfm

extern "C" int kdfm_gemm(const kdfm_gemm_desc* d, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(d != nullptr, "null descriptor");
  KDFM_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0, "negative size");
  KDFM_REQUIRE(d->batch1 >= 1 && d->batch2 >= 1, "batch must be >= 1");
  KDFM_REQUIRE(d->splitk >= 1 && d->splitk <= 4096, "splitk out of range");
  KDFM_REQUIRE(d->math == KDFM_MATH_F32 || d->math == KDFM_MATH_BF16, "bad math mode");
  if (d->M == 0 || d->N == 0) return KDFM_OK;
  KDFM_REQUIRE(d->A && d->B && d->C, "null operand");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_BIAS) || d->bias, "EPI_BIAS without bias");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_RESID) || d->R, "EPI_RESID without R");
  KDFM_REQUIRE(!(d->epi & (KDFM_EPI_DRELU | KDFM_EPI_DSILU)) || d->aux, "derivative epilogue without aux");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_STORE_PRE) || d->Cpre, "EPI_STORE_PRE without Cpre");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_DROPOUT) || (d->dropout_p >= 0.f && d->dropout_p < 1.f), "dropout p");
  KDFM_REQUIRE(d->splitk == 1 || (d->epi == KDFM_EPI_ATOMIC), "split-K requires the ATOMIC epilogue only");
  KDFM_REQUIRE((d->epi & KDFM_EPI_ATOMIC) == 0 || d->epi == KDFM_EPI_ATOMIC, "ATOMIC excludes other epilogues");
  if (d->amode == KDFM_LD_CONV || d->bmode == KDFM_LD_CONV)
    KDFM_REQUIRE(d->conv_c > 0 && d->conv_t > 0 && d->conv_taps > 0, "conv mode needs conv_c/conv_t/taps");
  KDFM_REQUIRE(!(d->amode == KDFM_LD_CONV && d->bmode == KDFM_LD_CONV), "only one CONV operand");
  P p{};   // value-initialised: fields a descriptor does not carry (partial, nseg, ...) start at 0
  p.A = d->A; p.B = d->B; p.C = d->C; p.bias = d->bias; p.R = d->R; p.aux = d->aux; p.Cpre = d->Cpre;
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.sAm = d->sAm; p.sAk = d->sAk; p.sBk = d->sBk; p.sBn = d->sBn; p.sCm = d->sCm; p.sCn = d->sCn;
  p.batch2 = d->batch2;
  p.bA1 = d->bA1; p.bA2 = d->bA2; p.bB1 = d->bB1; p.bB2 = d->bB2; p.bC1 = d->bC1; p.bC2 = d->bC2;
  p.alpha = d->alpha; p.beta = d->beta; p.rscale = d->rscale; p.dropout_p = d->dropout_p;
  p.seed = d->seed; p.rng_stream = d->rng_stream;
  p.epi = d->epi; p.splitk = d->splitk; p.taps = d->conv_taps; p.pad = d->conv_pad;
  p.conv_c = d->conv_c; p.conv_t = d->conv_t;
  p.mask_len = d->mask_len; p.mask_T = d->mask_T; p.mask_div = d->mask_div;
  p.loss_acc = d->loss_acc; p.loss_scale = d->loss_scale;
  p.ones_out = d->ones_out; p.ones_col = d->ones_col;
  p.ws = d->ws; p.ws_len = d->ws_len;
  p.Bh = d->Bh; p.sBh = d->sBh;
  if (d->ones_col >= 0)
    KDFM_REQUIRE(d->ones_out && (d->epi & KDFM_EPI_ATOMIC) && d->ones_col == d->N - 1 && d->batch1 == 1 &&
                     d->batch2 == 1,
                 "ones column needs ATOMIC, ones_out, ones_col == N-1 and an unbatched GEMM");
  if (d->epi & KDFM_EPI_ROWMASK)
    KDFM_REQUIRE(d->mask_len && d->mask_T > 0 && d->mask_div > 0 && d->batch1 == 1 && d->batch2 == 1,
                 "ROWMASK needs mask_len/mask_T/mask_div and an unbatched GEMM");
  if (d->epi & KDFM_EPI_MSE) KDFM_REQUIRE(d->loss_acc && d->R, "MSE needs loss_acc and target R");
  if (d->K == 0) p.splitk = 1;
  hipStream_t st = as_stream(stream);
  p.partial = 0;
  if (deterministic() && (d->epi & KDFM_EPI_ATOMIC)) {
    // fixed-order reductions: split-K partials go to the caller's workspace and are folded in split
    // order (or, without a workspace, no split: one add per output element per launch); a batch
    // axis that reduces into one C (a zero C batch stride) is walked by successive launches on the
    // stream instead of concurrent atomics
    const bool red1 = d->batch1 > 1 && d->bC1 == 0, red2 = d->batch2 > 1 && d->bC2 == 0;
    if (red1 || red2) {
      kdfm_gemm_desc e = *d;
      e.splitk = 1;
      const int64_t n1 = red1 ? d->batch1 : 1, n2 = red2 ? d->batch2 : 1;
      for (int64_t i1 = 0; i1 < n1; ++i1)
        for (int64_t i2 = 0; i2 < n2; ++i2) {
          e.A = d->A + i1 * (red1 ? d->bA1 : 0) + i2 * (red2 ? d->bA2 : 0);
          e.B = d->B + i1 * (red1 ? d->bB1 : 0) + i2 * (red2 ? d->bB2 : 0);
          e.batch1 = red1 ? 1 : d->batch1;
          e.batch2 = red2 ? 1 : d->batch2;
          const int rc = kdfm_gemm(&e, stream);
          if (rc) return rc;
        }
      return KDFM_OK;
    }
    const int64_t need = (int64_t)p.splitk * d->M * d->N;
    // the bf16 wide-tile / row-parallel weight-gradient kernels fold their partials in order themselves
    const bool wide = d->math == KDFM_MATH_BF16 && d->ws &&
                      (rowstream_wgrad_ws(p, d->amode, d->bmode, 1) > 0 || wgrad_rows_ws(p, d->amode, d->bmode, 1) > 0);
    if (p.splitk > 1 && d->batch1 * d->batch2 == 1 && d->ws && d->ws_len >= need && !wide) {
      p.partial = 1;
      set_route(ROUTE_SPLIT_FOLD);
      dim3 grid((unsigned)ceil_div(d->M, BM), (unsigned)ceil_div(d->N, BN), (unsigned)p.splitk);
      const int rc = d->math == KDFM_MATH_BF16 ? launch<true>(p, d->amode, d->bmode, grid, st)
                                               : launch<false>(p, d->amode, d->bmode, grid, st);
      if (rc) return rc;
      return launch_split_fold(p, p.splitk, true, st);
    }
    if (!wide) p.splitk = 1;
  }
  if (d->math == KDFM_MATH_BF16 && d->K > 0) {
    const int64_t batch = d->batch1 * d->batch2;
    int rc = try_wgrad_rows(p, d->amode, d->bmode, batch, st);
    if (rc >= 0) return set_route(ROUTE_WGRAD_ROWS), rc;
    rc = try_rowstream_wgrad(p, d->amode, d->bmode, batch, st);
    if (rc >= 0) return set_route(ROUTE_RS_WGRAD), rc;
    set_route(ROUTE_SKINNY);  // try_skinny_fwd marks its LDS-slab conv instance itself
    rc = try_skinny_fwd(p, d->amode, d->bmode, batch, st);
    if (rc >= 0) return rc;
    rc = try_rowstream_fwd(p, d->amode, d->bmode, batch, st);
    if (rc >= 0) return set_route(ROUTE_RS_FWD), rc;
  }
  set_route(ROUTE_GENERIC);
  const int64_t gx = ceil_div(d->M, BM), gy = ceil_div(d->N, BN), gz = d->batch1 * d->batch2 * p.splitk;
  KDFM_REQUIRE(gx < (1ll << 31) && gy < 65536 && gz < 65536, "grid too large");
  dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)gz);
  return d->math == KDFM_MATH_BF16 ? launch<true>(p, d->amode, d->bmode, grid, st)
                                   : launch<false>(p, d->amode, d->bmode, grid, st);
}

extern "C" int64_t kdfm_gemm_ws(const kdfm_gemm_desc* d) {
  using namespace kdfm;
  if (!d || d->K <= 0 || d->M <= 0 || d->N <= 0) return 0;
  if (d->math != KDFM_MATH_BF16 && !(deterministic() && (d->epi & KDFM_EPI_ATOMIC) && d->splitk > 1)) return 0;
  GemmP p{};
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.sAm = d->sAm; p.sAk = d->sAk; p.sBk = d->sBk; p.sBn = d->sBn; p.sCm = d->sCm; p.sCn = d->sCn;
  p.epi = d->epi; p.splitk = d->splitk; p.taps = d->conv_taps; p.pad = d->conv_pad;
  p.conv_c = d->conv_c; p.conv_t = d->conv_t; p.ones_col = d->ones_col; p.ones_out = d->ones_out;
  p.Bh = nullptr; p.sBh = 0;
  int64_t n = rowstream_wgrad_ws(p, d->amode, d->bmode, d->batch1 * d->batch2);
  if (d->math == KDFM_MATH_BF16) {
    const int64_t w = wgrad_rows_ws(p, d->amode, d->bmode, d->batch1 * d->batch2);
    if (w > n) n = w;
  }
  if (deterministic() && (d->epi & KDFM_EPI_ATOMIC) && d->splitk > 1 && d->batch1 * d->batch2 == 1) {
    const int64_t sk = (int64_t)d->splitk * d->M * d->N;  // ordered split-K partials
    if (sk > n) n = sk;
  }
  return n;
}
