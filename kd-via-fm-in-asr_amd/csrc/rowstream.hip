// Row-streaming GEMMs for the tall, narrow products of the ver5 step (bf16 MFMA, f32 accumulate).
//
// The KD heads run every 1x1 / k=3 conv of TeacherAutoEncoder, StudentProjector, NoiseAdapter,
// SimpleDenoiser and FlowMatchingModule (asr_train_diffm.py:400-497) over the stacked
// (16 layers x B x T') = 205,312 rows with only 96..176 output channels, and every Linear's weight
// gradient contracts over all rows.  The generic 64x64-tile kernel re-reads the streamed operand
// once per 64-wide N tile and wastes a third of each MFMA on N = 96.  Two specialised kernels:
//
//  rs_fwd    C[M x N] = epi(alpha * A * B) with N <= 16*NT.  The whole B (weights, <= ~80 KB bf16)
//            is resident in LDS for the life of a persistent workgroup; A is streamed in 64-row
//            tiles (4 waves x 16 rows, each wave computes 16 x N), the next tile's rows are
//            prefetched into registers while the MFMAs run.  CONV mode (k = tap*C + c, Conv1d k=3
//            along frames) stages ONE slab of 64 + taps - 1 rows and forms all taps from it, so
//            the activation is read from HBM exactly once.
//  rs_wgrad  C[M x N] += alpha * A^T B with K (rows) >> M*N: each workgroup owns a whole
//            (32*MT) x (32*NT) C tile in registers over a chunk of rows, streams both operands
//            once (double-buffered LDS, one barrier per 32-row step) and writes its f32 partial to
//            a workspace; a fold kernel adds alpha * sum(partials) into C (and the implicit ones
//            column -> bias gradient).  The A/B operands are read once instead of once per tile.
//
// Both are selected inside kdfm_gemm (bf16 math only; the f32 parity mode keeps the generic
// kernel) so every call site and the C-ABI stay unchanged.
#include "gemm_common.h"

#include <cstdlib>

namespace kdfm {
namespace {

constexpr int RS_NT = 256;   // threads per workgroup
constexpr int RS_BM = 64;    // rows per forward tile
constexpr int PRE_MAX = 12;  // float4 prefetch registers per thread (forward)

__device__ __forceinline__ void pack4_bf16(uint16_t* dst, float4 v) {
  const uint32_t lo = pack_bf16x2(v.x, v.y);
  const uint32_t hi = pack_bf16x2(v.z, v.w);
  *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
}

// ------------------------------------------------------------------------------------------
// rs_fwd: one 64-row tile per workgroup, small register/LDS footprint so 2-4 workgroups share a
// CU and hide each other's HBM latency (pure streaming: occupancy, not a deep per-block
// pipeline, is what keeps enough bytes in flight).  B is staged per K-chunk (one tap in CONV
// mode) from L2.  The epilogue loads every R/aux value it needs before the first store.
// ------------------------------------------------------------------------------------------
struct FwdGeo {
  int chunk;    // K per B stage (conv_c in CONV mode, Kp in KC mode)
  int nchunks;  // taps (CONV) or 1
  int lda;      // A image row stride (bf16)
  int ldb;      // B image row stride (bf16) = chunk + 8
  int arows;    // staged A rows (64, or 64 + taps - 1)
  int acols;    // staged A columns (K in KC mode, conv_c in CONV mode)
};

template <int NT, int AMODE, int APRE, int WV>
__global__ __launch_bounds__(64 * WV, (WV == 4) ? 2 : 1) void rs_fwd_kernel(GemmP p, FwdGeo g) {
  constexpr int NTH = 64 * WV;     // threads
  constexpr int TBM = 16 * WV;     // rows per tile
  extern __shared__ __attribute__((aligned(16))) uint16_t rs_lds[];
  uint16_t* As = rs_lds;                     // [arows][lda]
  uint16_t* Bs = rs_lds + g.arows * g.lda;   // [16*NT][ldb]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * TBM;

  // ---- A tile -> registers (issued first) ----
  const int cq = g.acols >> 2;
  const int atotal = g.arows * cq;
  float4 av[APRE];
#pragma unroll
  for (int i = 0; i < APRE; ++i) {
    const int q = threadIdx.x + i * NTH;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < atotal) {
      const int r = q / cq, c4 = (q - r * cq) * 4;
      const int64_t xr = (AMODE == KDFM_LD_CONV) ? m0 - p.pad + r : m0 + r;
      if (xr >= 0 && xr < p.M) v = *reinterpret_cast<const float4*>(p.A + xr * p.sAm + c4);
    }
    av[i] = v;
  }

  // ---- B chunk staging (fp32 L2 -> bf16 LDS), 8 float4 in flight per batch ----
  constexpr int NP = 16 * NT;
  auto stage_B = [&](int c) {
    const int k0 = c * g.chunk;
    if (p.sBk == 1) {  // W[n][k]
      const int kq = g.chunk >> 2;
      const int total = NP * kq;
      for (int base = 0; base < total; base += NTH * 8) {
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int e = base + threadIdx.x + i * NTH;
          const int n = e / kq, k = k0 + (e - n * kq) * 4;
          v[i] = (e < total && n < p.N && k < p.K) ? *reinterpret_cast<const float4*>(p.B + k + (int64_t)n * p.sBn)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int e = base + threadIdx.x + i * NTH;
          if (e < total) {
            const int n = e / kq, kk = (e - n * kq) * 4;
            pack4_bf16(Bs + n * g.ldb + kk, v[i]);
          }
        }
      }
    } else {           // B(k, n) contiguous along n
      constexpr int nq = NP / 4;
      const int total = g.chunk * nq;
      for (int base = 0; base < total; base += NTH * 8) {
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int e = base + threadIdx.x + i * NTH;
          const int kk = e / nq, n = (e - kk * nq) * 4;
          const int k = k0 + kk;
          v[i] = (e < total && n < p.N && k < p.K) ? *reinterpret_cast<const float4*>(p.B + (int64_t)k * p.sBk + n)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int e = base + threadIdx.x + i * NTH;
          if (e < total) {
            const int kk = e / nq, n = (e - kk * nq) * 4;
            Bs[(n + 0) * g.ldb + kk] = f2bf(v[i].x);
            Bs[(n + 1) * g.ldb + kk] = f2bf(v[i].y);
            Bs[(n + 2) * g.ldb + kk] = f2bf(v[i].z);
            Bs[(n + 3) * g.ldb + kk] = f2bf(v[i].w);
          }
        }
      }
    }
  };

  stage_B(0);
#pragma unroll
  for (int i = 0; i < APRE; ++i) {
    const int q = threadIdx.x + i * NTH;
    if (q < atotal) {
      const int r = q / cq, c4 = (q - r * cq) * 4;
      pack4_bf16(As + r * g.lda + c4, av[i]);
    }
  }
  if (AMODE == KDFM_LD_KC && g.acols < g.chunk) {  // K % 32 != 0: zero the k tail
    const int tail = g.chunk - g.acols;
    for (int e = threadIdx.x; e < g.arows * tail; e += NTH) {
      const int r = e / tail;
      As[r * g.lda + g.acols + (e - r * tail)] = 0;
    }
  }
  __syncthreads();

  const int rl = wave * 16 + (lane & 15);  // this lane's A row within the tile
  const int64_t m = m0 + rl;
  const int tfr = (AMODE == KDFM_LD_CONV) ? (int)(m % p.conv_t) : 0;
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < g.nchunks; ++c) {
    if (c > 0) {
      __syncthreads();  // all waves done with the previous B chunk
      stage_B(c);
      __syncthreads();
    }
    bool ok = true;
    int arow = rl;
    if constexpr (AMODE == KDFM_LD_CONV) {
      const int tt = tfr + c - p.pad;
      ok = m < p.M && tt >= 0 && tt < p.conv_t;
      arow = rl + c;
    }
    const uint16_t* ap = As + arow * g.lda + ((AMODE == KDFM_LD_CONV) ? 0 : c * g.chunk) + 8 * (lane >> 4);
    const uint16_t* bp = Bs + (lane & 15) * g.ldb + 8 * (lane >> 4);
    for (int ks = 0; ks < g.chunk; ks += 32) {
      const bf16x8 af = ok ? *reinterpret_cast<const bf16x8*>(ap + ks) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(bp + j * 16 * g.ldb + ks);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[j], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: operand loads first, then stores ----
  const int epi = p.epi;
  const uint64_t seed = (epi & KDFM_EPI_DROPOUT) ? load_seed(p.seed) : 0ull;
  const float keep_scale = (epi & KDFM_EPI_DROPOUT) ? 1.f / (1.f - p.dropout_p) : 1.f;
  float mse_part = 0.f;
  const int64_t mb = m0 + wave * 16 + (lane >> 4) * 4;
  const int nb = lane & 15;
  const float* pre_src = (epi & (KDFM_EPI_RESID | KDFM_EPI_MSE)) ? p.R
                         : (epi & (KDFM_EPI_DRELU | KDFM_EPI_DSILU)) ? p.aux : nullptr;
  if (pre_src && !(epi & (KDFM_EPI_BETA | KDFM_EPI_STORE_PRE)) &&
      !((epi & (KDFM_EPI_RESID | KDFM_EPI_MSE)) && (epi & (KDFM_EPI_DRELU | KDFM_EPI_DSILU)))) {
    // single side operand (R or aux): batch its loads
    float pv[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t mo = mb + r;
        const int n = j * 16 + nb;
        pv[j][r] = (mo < p.M && n < p.N) ? pre_src[mo * p.sCm + n * p.sCn] : 0.f;
      }
    const bool use_r = (epi & (KDFM_EPI_RESID | KDFM_EPI_MSE)) != 0;
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t mo = mb + r;
        const int n = j * 16 + nb;
        if (mo >= p.M || n >= p.N) continue;
        float v = p.alpha * acc[j][r];
        if (epi & KDFM_EPI_BIAS) v += p.bias[n];
        const int64_t off = mo * p.sCm + n * p.sCn;
        if (epi & KDFM_EPI_MSE) {
          const float diff = v - pv[j][r];
          mse_part += diff * diff;
          p.C[off] = p.rscale * diff;
          continue;
        }
        if (epi & KDFM_EPI_RELU) v = fmaxf(v, 0.f);
        if (epi & KDFM_EPI_SILU) v = siluf_(v);
        if (epi & KDFM_EPI_DROPOUT) {
          const uint64_t idx = (uint64_t)mo * (uint64_t)p.N + (uint64_t)n;
          v = dropout_keep(seed, p.rng_stream, idx, p.dropout_p) ? v * keep_scale : 0.f;
        }
        if (!use_r) {
          if (epi & KDFM_EPI_DRELU) v = (pv[j][r] > 0.f) ? v : 0.f;
          if (epi & KDFM_EPI_DSILU) v *= dsiluf_(pv[j][r]);
        } else {
          v = pv[j][r] + p.rscale * v;
        }
        if (epi & KDFM_EPI_ROWMASK) {
          const int64_t fr = mo / p.mask_div;
          const int64_t t = fr % p.mask_T, u = fr / p.mask_T;
          if (t >= p.mask_len[u]) v = 0.f;
        }
        p.C[off] = v;
      }
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t mo = mb + r;
        const int64_t n = j * 16 + nb;
        if (mo >= p.M || n >= p.N) continue;
        epilogue_store(p, 0, mo, n, mo * p.sCm + n * p.sCn, p.alpha * acc[j][r], seed, keep_scale, mse_part);
      }
  }
  if (epi & KDFM_EPI_MSE) {
    mse_part = wave_sum(mse_part);
    if (lane == 0) atomicAdd(p.loss_acc, mse_part * p.loss_scale);
  }
}

// ------------------------------------------------------------------------------------------
// rs_wgrad
// ------------------------------------------------------------------------------------------
constexpr int WG_LDK = 40;  // bf16 row stride of the [row][32 k] images

struct WgGeo {
  int64_t tilesN;
  int64_t kchunk;   // rows per split (multiple of 32)
  int64_t Nmem;     // columns present in B memory (N - 1 with a ones column, else N)
};

// One staging unit = 8 consecutive k rows x 2 consecutive columns (m for A, n for B): eight 8-byte
// row loads (coalesced across lanes), then per column one 16-byte LDS store of 8 k values into the
// [col][k] image (columns 2 apart across lanes -> at most 2-way bank conflicts).
template <int MT, int NT>
struct WgUnits {
  static constexpr int A = 4 * (32 * MT) / 2;  // (32/8) k-groups x (BMw/2) column pairs
  static constexpr int B = 4 * (32 * NT) / 2;
  static constexpr int PA = (A + RS_NT - 1) / RS_NT;
  static constexpr int PB = (B + RS_NT - 1) / RS_NT;
};

__device__ __forceinline__ float2 ld2_or0(const float* ptr, bool ok) {
  return ok ? *reinterpret_cast<const float2*>(ptr) : make_float2(0.f, 0.f);
}

// A(m, k) = A[k*sAk + m] (sAm == 1)
template <int MT>
__device__ __forceinline__ void wg_fetch_A(float2 (&v)[8], const GemmP& p, int u, int64_t m0, int64_t k0,
                                           int64_t kend) {
  constexpr int CG = (32 * MT) / 2;
  const int kg = u / CG, cg = u - kg * CG;
  const int64_t m = m0 + cg * 2;
  const bool mok = m < p.M;  // M even is required by the dispatcher
  const int64_t kb = k0 + kg * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = ld2_or0(p.A + (kb + i) * p.sAk + m, mok && kb + i < kend);
}

// B(k, n): XC -> B[k*sBk + n]; CONV -> X[(k + tap - pad)*sBk + c], n = tap*C + c.
template <bool BCONV, int NT>
__device__ __forceinline__ void wg_fetch_B(float2 (&v)[8], const GemmP& p, const WgGeo& g, int u, int64_t n0,
                                           int64_t k0, int64_t kend) {
  constexpr int CG = (32 * NT) / 2;
  const int kg = u / CG, cg = u - kg * CG;
  const int64_t n = n0 + cg * 2;
  const int64_t kb = k0 + kg * 8;
  if (n + 1 < g.Nmem) {
    if constexpr (BCONV) {
      const int C = (int)p.conv_c, T = (int)p.conv_t;
      const int tap = (int)n / C, c = (int)n - tap * C;
      int t = (int)((uint64_t)kb % (uint32_t)T);  // frame of row kb within its utterance
      const float* src = p.B + (kb + tap - p.pad) * p.sBk + c;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int tt = t + tap - p.pad;
        v[i] = ld2_or0(src + i * p.sBk, kb + i < kend && tt >= 0 && tt < T);
        t = (t + 1 == T) ? 0 : t + 1;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = ld2_or0(p.B + (kb + i) * p.sBk + n, kb + i < kend);
    }
    return;
  }
  // ragged edge / implicit ones column: element-wise
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t k = kb + i;
    float e[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t nn = n + q;
      float x = 0.f;
      if (k < kend) {
        if (nn == p.ones_col) {
          x = 1.f;
        } else if (nn < g.Nmem) {
          if constexpr (BCONV) {
            const int64_t tap = nn / p.conv_c, c = nn - tap * p.conv_c;
            const int64_t tt = (k % p.conv_t) + tap - p.pad;
            if (tt >= 0 && tt < p.conv_t) x = p.B[(k + tap - p.pad) * p.sBk + c];
          } else {
            x = p.B[k * p.sBk + nn];
          }
        }
      }
      e[q] = x;
    }
    v[i] = make_float2(e[0], e[1]);
  }
}

// Write one unit transposed into the [col][k] image: per column 8 k values -> one 16-byte store.
template <int COLS>
__device__ __forceinline__ void wg_store_unit(uint16_t* img, int u, const float2 (&v)[8]) {
  constexpr int CG = COLS / 2;
  const int kg = u / CG, cg = u - kg * CG;
  float t0[8], t1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    t0[i] = v[i].x;
    t1[i] = v[i].y;
  }
  const bf16x8 c0 = pack_bf16x8<bf16x8>(t0), c1 = pack_bf16x8<bf16x8>(t1);
  *reinterpret_cast<bf16x8*>(img + (cg * 2 + 0) * WG_LDK + kg * 8) = c0;
  *reinterpret_cast<bf16x8*>(img + (cg * 2 + 1) * WG_LDK + kg * 8) = c1;
}

template <int MT, int NT, bool BCONV>
__global__ __launch_bounds__(RS_NT, (MT * NT <= 18) ? 2 : 1) void rs_wgrad_kernel(GemmP p, WgGeo g) {
  using U = WgUnits<MT, NT>;
  constexpr int BMW = 32 * MT, BNW = 32 * NT;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BMW * WG_LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BNW * WG_LDK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t tm = blockIdx.x / g.tilesN, tn = blockIdx.x - tm * g.tilesN;
  const int64_t m0 = tm * BMW, n0 = tn * BNW;
  const int64_t split = blockIdx.y;
  const int64_t kb = split * g.kchunk;
  const int64_t ke = (kb + g.kchunk < p.K) ? kb + g.kchunk : p.K;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float2 ra[U::PA][8], rb[U::PB][8];
  auto fetch = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < U::PA; ++i) {
      const int u = threadIdx.x + i * RS_NT;
      if (u < U::A) wg_fetch_A<MT>(ra[i], p, u, m0, k0, ke);
    }
#pragma unroll
    for (int i = 0; i < U::PB; ++i) {
      const int u = threadIdx.x + i * RS_NT;
      if (u < U::B) wg_fetch_B<BCONV, NT>(rb[i], p, g, u, n0, k0, ke);
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < U::PA; ++i) {
      const int u = threadIdx.x + i * RS_NT;
      if (u < U::A) wg_store_unit<BMW>(As[buf], u, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < U::PB; ++i) {
      const int u = threadIdx.x + i * RS_NT;
      if (u < U::B) wg_store_unit<BNW>(Bs[buf], u, rb[i]);
    }
  };

  if (kb < ke) {
    fetch(kb);
    stage(0);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t k0 = kb; k0 < ke; k0 += 32) {
    const bool more = k0 + 32 < ke;
    if (more) fetch(k0 + 32);
    bf16x8 af[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(As[buf] + (wr * 16 * MT + i * 16 + (lane & 15)) * WG_LDK + 8 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const bf16x8 bfr =
          *reinterpret_cast<const bf16x8*>(Bs[buf] + (wc * 16 * NT + j * 16 + (lane & 15)) * WG_LDK + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
    }
    if (more) stage(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // partial tile -> ws[split][m][n]  (f32, unscaled)
  float* wsp = p.ws + split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * 16 * MT + i * 16 + (lane >> 4) * 4 + r;
        const int64_t n = n0 + wc * 16 * NT + j * 16 + (lane & 15);
        if (m < p.M && n < p.N) wsp[m * p.N + n] = acc[i][j][r];
      }
}

// C(m, n) += alpha * sum_s ws[s][m][n]   (n == ones_col -> ones_out[m]).  grid.y = split slabs.
__global__ __launch_bounds__(256) void rs_fold_kernel(GemmP p, int64_t S, int64_t per) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t MN = p.M * p.N;
  if (e >= MN) return;
  const int64_t s0 = (int64_t)blockIdx.y * per;
  const int64_t s1 = (s0 + per < S) ? s0 + per : S;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int64_t s = s0;
  for (; s + 3 < s1; s += 4) {
    a0 += p.ws[(s + 0) * MN + e];
    a1 += p.ws[(s + 1) * MN + e];
    a2 += p.ws[(s + 2) * MN + e];
    a3 += p.ws[(s + 3) * MN + e];
  }
  for (; s < s1; ++s) a0 += p.ws[s * MN + e];
  const float v = p.alpha * ((a0 + a1) + (a2 + a3));
  const int64_t m = e / p.N, n = e - m * p.N;
  if (n == p.ones_col)
    atomicAdd(p.ones_out + m, v);
  else
    atomicAdd(p.C + m * p.sCm + n * p.sCn, v);
}

// ---- instance selection ----
struct WgCfg { int mt, nt; };

bool wg_pick(int64_t M, int64_t N, WgCfg& c) {
  if (M <= 96) {
    c.mt = 3;
    const int64_t nt = ceil_div(N, 32);
    c.nt = nt <= 3 ? 3 : nt <= 4 ? 4 : nt <= 6 ? 6 : nt <= 10 ? 10 : 12;
  } else if (M <= 192) {
    c.mt = 6;
    const int64_t nt = ceil_div(N, 32);
    c.nt = nt <= 3 ? 3 : nt <= 4 ? 4 : 6;
  } else {
    c.mt = 12;
    c.nt = 3;
  }
  return true;
}

bool wg_eligible(const GemmP& p, int amode, int bmode, int64_t batch) {
  if (batch != 1 || p.epi != KDFM_EPI_ATOMIC || amode != KDFM_LD_XC) return false;
  if (p.sAm != 1 || (p.sAk & 1) || (p.M & 1) || (((uintptr_t)p.A) & 7)) return false;
  static const int64_t min_k = [] {
    const char* e = getenv("KDFM_RS_WGRAD_MINK");
    return e ? atoll(e) : 65536ll;
  }();
  if (p.K < min_k) return false;
  if (bmode == KDFM_LD_XC) {
    if (p.sBn != 1 || (p.sBk & 1) || (((uintptr_t)p.B) & 7)) return false;
  } else if (bmode == KDFM_LD_CONV) {
    if (p.sBn != 1 || (p.conv_c & 1) || (p.sBk & 1) || (((uintptr_t)p.B) & 7) || p.conv_t >= (1ll << 31)) return false;
  } else {
    return false;
  }
  if (p.ones_col >= 0 && p.ones_col != p.N - 1) return false;
  WgCfg c;
  wg_pick(p.M, p.N, c);
  if (bmode == KDFM_LD_CONV && !(c.mt == 3 && c.nt == 10)) return false;
  return true;
}

void wg_plan(const GemmP& p, int64_t& tiles, int64_t& tilesN, int64_t& S, int64_t& kchunk, WgCfg& c) {
  wg_pick(p.M, p.N, c);
  const int64_t tilesM = ceil_div(p.M, 32 * c.mt);
  tilesN = ceil_div(p.N, 32 * c.nt);
  tiles = tilesM * tilesN;
  const int64_t steps = ceil_div(p.K, 32);
  static const int64_t target = [] {
    const char* e = getenv("KDFM_RS_WGRAD_WGS");
    return e ? atoll(e) : 256ll;
  }();
  S = target / tiles;
  if (S < 1) S = 1;
  static const int64_t min_steps = [] {
    const char* e = getenv("KDFM_RS_WGRAD_STEPS");
    return e ? atoll(e) : 4ll;
  }();
  const int64_t smax = steps / min_steps > 0 ? steps / min_steps : 1;
  if (S > smax) S = smax;
  kchunk = ceil_div(steps, S) * 32;
  S = ceil_div(p.K, kchunk);
}

template <int MT, int NT, bool BCONV>
int launch_wg(const GemmP& p, const WgGeo& g, int64_t tiles, int64_t S, hipStream_t st) {
  hipLaunchKernelGGL((rs_wgrad_kernel<MT, NT, BCONV>), dim3((unsigned)tiles, (unsigned)S), dim3(RS_NT), 0, st, p, g);
  return check_launch("kdfm_gemm(rowstream wgrad)");
}

}  // namespace

int64_t rowstream_wgrad_ws(const GemmP& p, int amode, int bmode, int64_t batch) {
  GemmP q = p;
  q.A = reinterpret_cast<const float*>(16);  // alignment checks only
  q.B = reinterpret_cast<const float*>(16);
  if (!wg_eligible(q, amode, bmode, batch)) return 0;
  int64_t tiles, tilesN, S, kchunk;
  WgCfg c;
  wg_plan(p, tiles, tilesN, S, kchunk, c);
  return S * p.M * p.N;
}

int try_rowstream_wgrad(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st) {
  if (!p.ws || !wg_eligible(p, amode, bmode, batch)) return -1;
  int64_t tiles, tilesN, S, kchunk;
  WgCfg c;
  wg_plan(p, tiles, tilesN, S, kchunk, c);
  if (p.ws_len < S * p.M * p.N) return -1;
  WgGeo g;
  g.tilesN = tilesN;
  g.kchunk = kchunk;
  g.Nmem = p.ones_col >= 0 ? p.ones_col : p.N;
  int rc;
  if (bmode == KDFM_LD_CONV) {
    rc = launch_wg<3, 10, true>(p, g, tiles, S, st);
  } else {
    switch (c.mt * 100 + c.nt) {
      case 303: rc = launch_wg<3, 3, false>(p, g, tiles, S, st); break;
      case 304: rc = launch_wg<3, 4, false>(p, g, tiles, S, st); break;
      case 306: rc = launch_wg<3, 6, false>(p, g, tiles, S, st); break;
      case 310: rc = launch_wg<3, 10, false>(p, g, tiles, S, st); break;
      case 312: rc = launch_wg<3, 12, false>(p, g, tiles, S, st); break;
      case 603: rc = launch_wg<6, 3, false>(p, g, tiles, S, st); break;
      case 604: rc = launch_wg<6, 4, false>(p, g, tiles, S, st); break;
      case 606: rc = launch_wg<6, 6, false>(p, g, tiles, S, st); break;
      default: rc = launch_wg<12, 3, false>(p, g, tiles, S, st); break;
    }
  }
  if (rc) return rc;
  return launch_split_fold(p, S, deterministic(), st);
}

int launch_split_fold(const GemmP& p, int64_t S, bool ordered, hipStream_t st) {
  const int64_t MN = p.M * p.N;
  const int64_t per = ordered ? S : 16;  // ordered: one fold thread sums every slab in order
  const int64_t slabs = ceil_div(S, per);
  hipLaunchKernelGGL(rs_fold_kernel, dim3((unsigned)ceil_div(MN, 256), (unsigned)slabs), dim3(256), 0, st, p, S, per);
  return check_launch("kdfm_gemm(split fold)");
}

namespace {
template <int NT, int AMODE, int APRE, int WV>
int launch_fwd(const GemmP& p, const FwdGeo& g, size_t lds, hipStream_t st) {
  const int64_t ntiles = ceil_div(p.M, 16 * WV);
  hipLaunchKernelGGL((rs_fwd_kernel<NT, AMODE, APRE, WV>), dim3((unsigned)ntiles), dim3(64 * WV), lds, st, p, g);
  return check_launch("kdfm_gemm(rowstream fwd)");
}
}  // namespace

int try_rowstream_fwd(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st) {
  if (batch != 1 || p.splitk != 1 || (p.epi & KDFM_EPI_ATOMIC) || p.ones_col >= 0) return -1;
  if (p.M < 16384 || p.N > 176) return -1;
  if (bmode != KDFM_LD_KC && bmode != KDFM_LD_XC) return -1;
  if (p.sBk == 1) {
    if ((p.sBn & 3) || (p.K & 3)) return -1;
  } else if (p.sBn == 1) {
    if ((p.sBk & 3) || (p.N & 3)) return -1;
  } else {
    return -1;
  }
  if (((uintptr_t)p.B) & 15) return -1;
  if (p.sAk != 1 || (p.sAm & 3) || (((uintptr_t)p.A) & 15)) return -1;
  static const int env_wv = [] {
    const char* e = getenv("KDFM_RS_CONV_WAVES");
    return e ? atoi(e) : 8;
  }();
  FwdGeo g;
  int wv = 4;
  if (amode == KDFM_LD_CONV) {
    if (p.conv_c % 32 != 0 || p.conv_c > 128 || p.K != p.taps * p.conv_c || p.pad < 0 || p.pad >= p.taps)
      return -1;
    wv = env_wv == 4 ? 4 : 8;
    g.chunk = (int)p.conv_c;
    g.nchunks = p.taps;
    g.arows = 16 * wv + p.taps - 1;
    g.acols = (int)p.conv_c;
    g.lda = g.acols + 8;
  } else if (amode == KDFM_LD_KC) {
    if ((p.K & 3) || p.K > 192) return -1;
    g.chunk = (int)ceil_div(p.K, 32) * 32;
    g.nchunks = 1;
    g.arows = 16 * wv;
    g.acols = (int)p.K;
    g.lda = g.chunk + 8;
  } else {
    return -1;
  }
  g.ldb = g.chunk + 8;
  const int apre = (int)ceil_div(g.arows * (g.acols / 4), 64 * wv);
  if (apre > 12) return -1;
  const int nt = p.N <= 96 ? 6 : 11;
  const size_t lds = (size_t)(g.arows * g.lda + 16 * nt * g.ldb) * sizeof(uint16_t);
  if (lds > 64 * 1024) return -1;
  if (amode == KDFM_LD_CONV) {
    if (nt != 6 || apre > 8) return -1;
    return wv == 8 ? launch_fwd<6, KDFM_LD_CONV, 8, 8>(p, g, lds, st) : launch_fwd<6, KDFM_LD_CONV, 8, 4>(p, g, lds, st);
  }
  if (nt == 6)
    return apre <= 8 ? launch_fwd<6, KDFM_LD_KC, 8, 4>(p, g, lds, st) : launch_fwd<6, KDFM_LD_KC, 12, 4>(p, g, lds, st);
  if (apre > 8) return -1;
  return launch_fwd<11, KDFM_LD_KC, 8, 4>(p, g, lds, st);
}

}  // namespace kdfm
