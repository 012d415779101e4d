// Striding ConvSubsampling forward as two fused kernels (bf16 MFMA mode).
//
// Reference: ConvSubsampling(subsampling='striding', factor 4, conv_channels = d), built
// conformer_encoder.py:381-390 and called :635 (source absent):
//   x (B,T,80) -> Conv2d(1->C, 3x3, s2, p1) -> ReLU -> Conv2d(C->C, 3x3, s2, p1) -> ReLU
// with padded frames masked to zero before each conv (A.3 flag, default on).
//
// The im2col formulation materialises 9x the conv1 output (1.6 GB for the teacher at B=32, 16 s)
// and streams it through a GEMM.  Here:
//   ss_conv1  y1 = mask1(ReLU(conv1(mask0(mel)))) computed directly (9 FMAs per output, K = 9 is
//             far too small for MFMA), stored channels-last as bf16 — the next kernel's MFMA
//             operand — and optionally as f32 for the backward;
//   ss_conv2  implicit GEMM: M = output positions (b,t2,f2), N = C_out, K = 9 taps x C_in.
//             A fragments are 16-byte loads of 8 consecutive channels of y1 at the tap's shifted
//             position (no im2col matrix); the tap's weight slab [C_out][C_in] (bf16, prepared
//             by ss_wprep) is double-buffered through LDS with one barrier per tap; 8 waves x 32
//             positions per workgroup, v_mfma_f32_32x32x16_bf16; bias + ReLU + len2 frame mask
//             fused in the epilogue, output channels-last f32 rows (b,t2,f2) x C — the layout the
//             following Linear(C*F2 -> d) consumes.
#include "common.h"

namespace kdfm {
namespace {

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// ---- weight prep: W (C, C, 3, 3) f32 -> wb[n][tap][ci] bf16, n < Np (zero rows >= C), ci < Cp
__global__ __launch_bounds__(256) void ss_wprep_kernel(const float* __restrict__ W, uint16_t* __restrict__ wb, int C,
                                                       int Np, int Cp) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)Np * 9 * Cp;
  if (idx >= total) return;
  const int ci = (int)(idx % Cp), tap = (int)((idx / Cp) % 9), n = (int)(idx / (9 * Cp));
  float v = 0.f;
  if (n < C && ci < C) v = W[((int64_t)n * C + ci) * 9 + tap];
  wb[idx] = f2bf(v);
}

// ---- conv1 + ReLU + masks: one thread = one output position x 8 channels
__global__ __launch_bounds__(256) void ss_conv1_kernel(const float* __restrict__ mel, const int64_t* __restrict__ mel_len,
                                                       const int64_t* __restrict__ len1, const float* __restrict__ w0,
                                                       const float* __restrict__ b0, uint16_t* __restrict__ y1b,
                                                       float* __restrict__ y1f, int B, int Tm, int F, int C, int T1,
                                                       int F1) {
  // weights and biases staged in LDS (C <= 256); 32-bit index math (B T1 F1 C/8 < 2^31, host-checked)
  __shared__ float ws[256 * 9], bs[256];
  for (int e = threadIdx.x; e < C * 9; e += 256) ws[e] = w0[e];
  for (int e = threadIdx.x; e < C; e += 256) bs[e] = b0[e];
  __syncthreads();
  const int CG = C >> 3;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  const uint32_t total = (uint32_t)B * T1 * F1 * CG;
  if (idx >= total) return;
  const int cg = (int)(idx % CG);
  const uint32_t pos32 = idx / CG;
  const int64_t pos = pos32;
  const int f1 = (int)(pos32 % F1);
  const int t1 = (int)((pos32 / F1) % T1);
  const int b = (int)(pos32 / ((uint32_t)F1 * T1));
  const int64_t ml = mel_len ? mel_len[b] : Tm;
  const bool rowok = !len1 || t1 < len1[b];
  float x[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int t = 2 * t1 - 1 + ky, f = 2 * f1 - 1 + kx;
      x[ky * 3 + kx] = (t >= 0 && t < Tm && t < ml && f >= 0 && f < F) ? mel[((int64_t)b * Tm + t) * F + f] : 0.f;
    }
  float out[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    float v = bs[c];
#pragma unroll
    for (int q = 0; q < 9; ++q) v = fmaf(ws[c * 9 + q], x[q], v);
    v = fmaxf(v, 0.f);
    out[j] = rowok ? v : 0.f;
  }
  *reinterpret_cast<bf16x8_t*>(y1b + pos * C + cg * 8) = pack_bf16x8<bf16x8_t>(out);
  if (y1f) {
    float4* d = reinterpret_cast<float4*>(y1f + pos * C + cg * 8);
    d[0] = make_float4(out[0], out[1], out[2], out[3]);
    d[1] = make_float4(out[4], out[5], out[6], out[7]);
  }
}

// ---- conv2 implicit GEMM
constexpr int SS_WAVES = 8;
constexpr int SS_NT = 64 * SS_WAVES;

struct SsGeo {
  int B, T1, F1, C, T2, F2;
  int64_t P;     // output positions B*T2*F2
  int Cp;        // C_in padded to 16 (k per tap)
  int ldb;       // LDS image row stride (Cp + 8)
};

// NCT 32-col tiles of C_out per wave, NWN waves across C_out, KS = Cp/16 k-steps per tap
template <int NCT, int NWN, int KS>
__global__ __launch_bounds__(SS_NT, 1) void ss_conv2_kernel(const uint16_t* __restrict__ y1, const int64_t* __restrict__ len2,
                                                             const uint16_t* __restrict__ wb, const float* __restrict__ b2,
                                                             float* __restrict__ y2, SsGeo g) {
  constexpr int NP = 32 * NCT * NWN;                    // padded C_out rows of the image
  constexpr int BMW = 32 * SS_WAVES / NWN;             // positions per workgroup tile
  extern __shared__ __attribute__((aligned(16))) uint16_t ss_lds[];
  const int ldb = g.ldb;
  uint16_t* buf0 = ss_lds;
  uint16_t* buf1 = ss_lds + NP * ldb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave / NWN, wn = wave % NWN;
  const int64_t pos0 = (int64_t)blockIdx.x * BMW + wm * 32;
  const int nb0 = wn * 32 * NCT;                       // first C_out column of this wave

  // this lane's A position (row r of the wave tile)
  const int64_t pa = pos0 + r;
  const bool pok = pa < g.P;
  const int f2 = pok ? (int)(pa % g.F2) : 0;
  const int t2 = pok ? (int)((pa / g.F2) % g.T2) : 0;
  const int bb = pok ? (int)(pa / ((int64_t)g.F2 * g.T2)) : 0;
  const uint16_t* ybase = y1 + (int64_t)bb * g.T1 * g.F1 * g.C;

  // B slab staging: NP rows x Cp bf16 per tap, 16-byte chunks
  constexpr int CPR = KS * 2;                           // 16-B chunks per row (Cp / 8)
  constexpr int CHUNKS = NP * CPR;
  constexpr int BPT = (CHUNKS + SS_NT - 1) / SS_NT;     // chunks per thread
  bf16x8_t breg[BPT];
  auto load_B = [&](int tap) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int e = threadIdx.x + i * SS_NT;
      if (e < CHUNKS) {
        const int n = e / CPR, q = e - n * CPR;
        breg[i] = *reinterpret_cast<const bf16x8_t*>(wb + ((int64_t)n * 9 + tap) * g.Cp + q * 8);
      }
    }
  };
  auto store_B = [&](uint16_t* dst) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int e = threadIdx.x + i * SS_NT;
      if (e < CHUNKS) {
        const int n = e / CPR, q = e - n * CPR;
        *reinterpret_cast<bf16x8_t*>(dst + n * ldb + q * 8) = breg[i];
      }
    }
  };
  auto load_A = [&](bf16x8_t (&a)[KS], int tap) {
    const int ky = tap / 3, kx = tap - ky * 3;
    const int t1 = 2 * t2 - 1 + ky, f1 = 2 * f2 - 1 + kx;
    const bool ok = pok && t1 >= 0 && t1 < g.T1 && f1 >= 0 && f1 < g.F1;
    const uint16_t* src = ybase + ((int64_t)t1 * g.F1 + f1) * g.C;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int ci = 16 * s + 8 * h;
      if (ok && ci < g.C)
        a[s] = *reinterpret_cast<const bf16x8_t*>(src + ci);
      else
        a[s] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };

  f32x16_t acc[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  bf16x8_t acur[KS], anxt[KS];
  load_B(0);
  load_A(acur, 0);
  store_B(buf0);
  __syncthreads();
  for (int tap = 0; tap < 9; ++tap) {
    const bool more = tap + 1 < 9;
    if (more) {
      load_B(tap + 1);
      load_A(anxt, tap + 1);
    }
    const uint16_t* bs = (tap & 1) ? buf1 : buf0;
    const uint16_t* bp = bs + (nb0 + r) * ldb + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
        const bf16x8_t bfr = *reinterpret_cast<const bf16x8_t*>(bp + j * 32 * ldb + 16 * s);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[s], bfr, acc[j], 0, 0, 0);
      }
    }
    if (more) {
      store_B((tap & 1) ? buf0 : buf1);
#pragma unroll
      for (int s = 0; s < KS; ++s) acur[s] = anxt[s];
    }
    __syncthreads();
  }

  // ---- epilogue: bias + ReLU + frame mask (t2 >= len2[b] -> 0); all loads before stores
  float bn[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) {
    const int n = nb0 + 32 * j + r;
    bn[j] = n < g.C ? b2[n] : 0.f;
  }
  bool rowok[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t pm = pos0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    bool ok = pm < g.P;
    if (ok && len2) {
      const int tt = (int)((pm / g.F2) % g.T2);
      const int b = (int)(pm / ((int64_t)g.F2 * g.T2));
      ok = tt < len2[b];
      rowok[i] = ok;
    } else {
      rowok[i] = ok;
    }
  }
#pragma unroll
  for (int j = 0; j < NCT; ++j) {
    const int n = nb0 + 32 * j + r;
    if (n >= g.C) continue;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t pm = pos0 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (pm >= g.P) continue;
      const float v = fmaxf(acc[j][i] + bn[j], 0.f);
      y2[pm * g.C + n] = rowok[i] ? v : 0.f;
    }
  }
}

template <int NCT, int NWN, int KS>
int ss_launch(const uint16_t* y1, const int64_t* len2, const uint16_t* wb, const float* b2, float* y2,
              const SsGeo& g, hipStream_t st) {
  const size_t lds = (size_t)2 * 32 * NCT * NWN * g.ldb * sizeof(uint16_t);
  if (lds > 64 * 1024) {
    static bool once = [] {
      hipFuncSetAttribute((const void*)ss_conv2_kernel<NCT, NWN, KS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024);
      return true;
    }();
    (void)once;
  }
  const int64_t grid = ceil_div(g.P, 32 * SS_WAVES / NWN);
  hipLaunchKernelGGL((ss_conv2_kernel<NCT, NWN, KS>), dim3((unsigned)grid), dim3(SS_NT), lds, st, y1, len2, wb, b2, y2, g);
  return check_launch("kdfm_subsample_conv2");
}


// ---- conv2 data gradient (transposed conv) without the im2col matrix --------------------------
// dy1[b,t1,f1,ci] = [y1 > 0] * sum_{ky,kx,co: 2 t2 - 1 + ky = t1, 2 f2 - 1 + kx = f1} W[co,ci,ky,kx] dy2[b,t2,f2,co]
// The input positions split into 4 parity classes (t1 % 2, f1 % 2) with a FIXED tap set each:
// t1 even takes ky = 1 (t2 = t1/2); t1 odd takes ky = 0 (t2 = (t1+1)/2) and ky = 2 (t2 = (t1-1)/2);
// the same for f1 / kx -> 1, 2, 2 or 4 taps.  Each workgroup computes 256 positions of one class as an
// implicit GEMM (M = positions, N = C_in, K = taps x C_out, v_mfma_f32_32x32x16_bf16): the class's
// tap weight slabs [ci][co] (bf16, prepared by ss_dgrad_wprep) are staged in LDS once, A fragments
// are 8 consecutive C_out of dy2 at the tap's source position (two float4 loads, converted), and the
// ReLU' of the conv1 output is applied in the epilogue.  Replaces linear_dx into a 9C-wide column
// matrix (813 MB at the bench shape) plus its col2im gather.
constexpr int SD_TPW = 4;   // position tiles per workgroup (amortises the tap-slab staging)

struct SdGeo {
  int B, T1, F1, C, T2, F2, Cp, ldb;
  int64_t npos[4];   // positions per class (class = 2 * (t1 % 2) + f1 % 2)
  int64_t wg0[5];    // first workgroup of each class; wg0[4] = grid size
  // fused conv0 weight gradient (wpart != null): conv0 = Conv2d(1 -> C, 3x3, stride 2, pad) over the
  // (B, Tm, Fm) mel frames (rows t >= mel_len[b] read as 0); per-workgroup partials
  // wpart[wg][C * 9 + C] = (sum dy1 x_patch | sum dy1), folded in workgroup order on the host side
  const float* mel; const int64_t* mel_len; int Tm, Fm, pad; float* wpart;
  const uint16_t* wt;   // tap slabs [tap][ci (Np)][co (Cp)] bf16 (ss_dgrad_wprep)
  int ldy;              // y1 row stride (elements, >= C: the fused forward's padded rows)
};

__global__ __launch_bounds__(256) void ss_dgrad_wprep_kernel(const float* __restrict__ W, uint16_t* __restrict__ wt,
                                                             int C, int Np, int Cp) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)9 * Np * Cp;
  if (idx >= total) return;
  const int co = (int)(idx % Cp), ci = (int)((idx / Cp) % Np), tap = (int)(idx / ((int64_t)Np * Cp));
  float v = 0.f;
  if (ci < C && co < C) v = W[((int64_t)co * C + ci) * 9 + tap];
  wt[idx] = f2bf(v);
}

// Per parity class (PT, PF) the taps are compile-time constants.  A wave owns 32 positions per tile:
// lane r (both halves) decodes position r ONCE per tile into per-wave LDS (its y1 row index and, with
// the fused conv0 weight gradient, its 9 mel patch values + the ones column), so the epilogue reads
// them as LDS broadcasts instead of re-deriving them per accumulator row.  dy2 / y1 / dy1 go through
// buffer descriptors (32-bit offsets; an out-of-range offset reads 0 / drops the store, which is how
// masked positions, padded channels and positions past the end are handled without branches), and
// tap 0's dy2 fragments are in flight while the ReLU' masks load.  (A next-tap prefetch spilled at 256
// VGPRs; with 227 and 8 waves per CU, the other wave of a SIMD covers the tap loads.)  (The previous form kept
// the taps in a runtime-indexed private array and re-decoded every accumulator row's position and
// mel patch per lane: ~3.4k VALU instructions per 32-position tile, ~600 us at the bench shape.)
constexpr int SD_PTS = 12;          // patch row stride (floats): 9 taps, the ones column, 2 pad
constexpr uint32_t SD_OOB = 0x7fffffffu;

template <int NCT, int KS>
struct SdFrag {
  float4 v[KS][2];
};

template <int NCT, int KS, int PT, int PF, bool DBF>
__device__ __forceinline__ void sd_class(const SdGeo& g, __amdgpu_buffer_rsrc_t rdy2, __amdgpu_buffer_rsrc_t ry1,
                                         __amdgpu_buffer_rsrc_t rdy1, bool has_dy1, uint16_t* lds, int cls,
                                         float (&wacc)[NCT][10]) {
  constexpr int NP = 32 * NCT;
  constexpr int CP = 16 * KS;
  constexpr int DT = PT ? 2 : 1, DF = PF ? 2 : 1, NTAP = DT * DF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nT = (g.T1 - PT + 1) / 2, nF = (g.F1 - PF + 1) / 2;
  // stage the class's tap slabs [t][ci][co] (row stride ldb)
  constexpr int cpr = CP / 8;
#pragma unroll
  for (int t = 0; t < NTAP; ++t) {
    const int ky = PT ? 2 * (t / DF) : 1, kx = PF ? 2 * (t % DF) : 1;
    const uint16_t* src = g.wt + (int64_t)(3 * ky + kx) * NP * CP;
    for (int e = threadIdx.x; e < NP * cpr; e += SS_NT) {
      const int row = e / cpr, c8 = (e - row * cpr) * 8;
      *reinterpret_cast<bf16x8_t*>(lds + (t * NP + row) * g.ldb + c8) =
          *reinterpret_cast<const bf16x8_t*>(src + (int64_t)row * CP + c8);
    }
  }
  __syncthreads();
  // per-wave LDS: patches [32][SD_PTS] f32, then y1 row indices [32] int
  float* pt = reinterpret_cast<float*>(lds + NTAP * NP * g.ldb) + wave * (32 * SD_PTS + 32);
  int* mp = reinterpret_cast<int*>(pt + 32 * SD_PTS);
  const int per_b = nT * nF;
  const int npos = (int)g.npos[cls];
  const int ntile = (npos + 32 * SS_WAVES - 1) / (32 * SS_WAVES);
  const int tile0 = (int)(blockIdx.x - g.wg0[cls]) * SD_TPW;
  const int tend = min(tile0 + SD_TPW, ntile);
  // lane's channel offsets (bytes) into dy2 rows per k-step s; padded channels (>= C) read out of range.
  // DBF: dy2 is bf16 (one 16-byte load of 8 channels per k-step, no conversion), else f32 (two, packed)
  constexpr uint32_t EB = DBF ? 2u : 4u;
  uint32_t coff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int co = 16 * s + 8 * h;
    coff[s] = co < g.C ? (uint32_t)co * EB : SD_OOB;
  }
  auto load_tap = [&](SdFrag<NCT, KS>& f, int t, bool ok, int b, int i, int j) {
    const int t2 = i + ((PT && (t / DF) == 0) ? 1 : 0), f2 = j + ((PF && (t % DF) == 0) ? 1 : 0);
    const bool in = ok && t2 < g.T2 && f2 < g.F2;
    const uint32_t base = in ? (uint32_t)(((b * g.T2 + t2) * g.F2 + f2) * g.C) * EB : SD_OOB;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint32_t o = (base == SD_OOB || coff[s] == SD_OOB) ? SD_OOB : base + coff[s];
      f.v[s][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rdy2, o, 0, 0));
      if constexpr (!DBF)
        f.v[s][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rdy2, o == SD_OOB ? SD_OOB : o + 16, 0, 0));
    }
  };
  SdFrag<NCT, KS> fa;   // a tap's dy2 fragments (f32); tap 0's are loaded before the ReLU' masks
  for (int tile = tile0; tile < tend; ++tile) {
    const int pos0 = tile * (32 * SS_WAVES) + wave * 32;
    // this lane's position (lanes r and r + 32 hold the same one)
    const int pa = pos0 + r;
    const bool ok = pa < npos;
    int b = 0, i = 0, j = 0;
    if (ok) {
      b = pa / per_b;
      const int rem = pa - b * per_b;
      i = rem / nF;
      j = rem - i * nF;
    }
    load_tap(fa, 0, ok, b, i, j);
    // keep the tap-0 loads here, ahead of the mask loads: left alone the scheduler sinks each load next to
    // its MFMA and waits for it there (one HBM round trip per fragment)
    __builtin_amdgcn_sched_barrier(0);
    const int t1 = 2 * i + PT, f1 = 2 * j + PF;
    if (h == 0) {
      mp[r] = ok ? (b * g.T1 + t1) * g.F1 + f1 : -1;
      if (g.wpart) {
        const int t0 = 2 * t1 - g.pad, f0 = 2 * f1 - g.pad;
        // every load unconditional at a clamped index and masked by a multiply: a conditional load is
        // branched around and waited for one at a time (9 serialized HBM round trips per tile)
        const int tl = !ok ? 0 : (g.mel_len ? (int)min((int64_t)g.Tm, g.mel_len[b]) : g.Tm);
        const float* mb = g.mel + (int64_t)b * g.Tm * g.Fm;
        float xp[SD_PTS];
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const int tt = t0 + tp / 3, ff = f0 + tp % 3;
          const bool in = tt >= 0 && tt < tl && ff >= 0 && ff < g.Fm;
          const float x = mb[in ? tt * g.Fm + ff : 0];
          xp[tp] = (in ? 1.f : 0.f) * x;
        }
        xp[9] = ok ? 1.f : 0.f;
        xp[10] = xp[11] = 0.f;
#pragma unroll
        for (int q = 0; q < SD_PTS / 4; ++q)
          *reinterpret_cast<float4*>(pt + r * SD_PTS + 4 * q) = make_float4(xp[4 * q], xp[4 * q + 1], xp[4 * q + 2], xp[4 * q + 3]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS writes land before its reads
    __builtin_amdgcn_wave_barrier();
    // y1 row indices of the accumulator rows (positions 8 (e / 4) + 4 h + e % 4) and their ReLU' masks
    auto rows4 = [&](int q) { return *reinterpret_cast<const int4*>(mp + 8 * q + 4 * h); };
    uint32_t mask[NCT];
    const uint32_t ldy2 = 2u * (uint32_t)g.ldy;   // y1 row stride in bytes
#pragma unroll
    for (int n = 0; n < NCT; ++n) mask[n] = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 v = rows4(q);
      const int mq[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int n = 0; n < NCT; ++n) {
        const int ci = 32 * n + r;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t o = (mq[u] >= 0 && ci < g.C) ? (uint32_t)mq[u] * ldy2 + 2u * (uint32_t)ci : SD_OOB;
          const uint16_t yb = __builtin_amdgcn_raw_buffer_load_b16(ry1, o, 0, 0);
          mask[n] |= ((yb & 0x7fff) != 0 && !(yb & 0x8000)) ? (1u << (4 * q + u)) : 0u;   // ReLU' from the bf16 sign
        }
      }
    }
    f32x16_t acc[NCT];
#pragma unroll
    for (int n = 0; n < NCT; ++n)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[n][e] = 0.f;
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      if (t > 0) {
        load_tap(fa, t, ok, b, i, j);
        __builtin_amdgcn_sched_barrier(0);   // all of the tap's loads issued before the first wait
      }
      bf16x8_t a[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if constexpr (DBF) {
          a[s] = __builtin_bit_cast(bf16x8_t, fa.v[s][0]);
        } else {
          const float q[8] = {fa.v[s][0].x, fa.v[s][0].y, fa.v[s][0].z, fa.v[s][0].w,
                              fa.v[s][1].x, fa.v[s][1].y, fa.v[s][1].z, fa.v[s][1].w};
          a[s] = pack_bf16x8<bf16x8_t>(q);
        }
      }
      const uint16_t* bp = lds + (t * NP + r) * g.ldb + 8 * h;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int n = 0; n < NCT; ++n) {
          const bf16x8_t bv = *reinterpret_cast<const bf16x8_t*>(bp + n * 32 * g.ldb + 16 * s);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], bv, acc[n], 0, 0, 0);
        }
    }
    // epilogue: dy1 = ReLU'(y1) * acc; stores dropped for masked rows / padded channels
#pragma unroll
    for (int n = 0; n < NCT; ++n)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[n][e] = ((mask[n] >> e) & 1u) ? acc[n][e] : 0.f;
    if (has_dy1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int4 v = rows4(q);
        const int mq[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int n = 0; n < NCT; ++n) {
          const int ci = 32 * n + r;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t o = (mq[u] >= 0 && ci < g.C) ? (uint32_t)(mq[u] * g.C + ci) * 4u : SD_OOB;
            // through a scalar temporary: hipcc (ROCm 7.2) lowers __builtin_bit_cast of an ext-vector
            // ELEMENT lvalue to element 0 whatever the index (tools/ss_dgrad_debug.py found it)
            const float val = acc[n][4 * q + u];
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, val), rdy1, o, 0, 0);
          }
        }
      }
    }
    if (g.wpart) {
      // conv0 weight gradient: wacc[n][tap] += dy1 x_patch[tap] over the tile's rows (patch rows are
      // LDS broadcasts within each half-wave)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float* pr = pt + (8 * (e >> 2) + 4 * h + (e & 3)) * SD_PTS;
        const float4 x0 = *reinterpret_cast<const float4*>(pr);
        const float4 x1 = *reinterpret_cast<const float4*>(pr + 4);
        const float2 x2 = *reinterpret_cast<const float2*>(pr + 8);
        const float xv[10] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w, x2.x, x2.y};
#pragma unroll
        for (int n = 0; n < NCT; ++n)
#pragma unroll
          for (int k = 0; k < 10; ++k) wacc[n][k] = fmaf(acc[n][e], xv[k], wacc[n][k]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // patch / index reads done before the next tile's writes
    __builtin_amdgcn_wave_barrier();
  }
}

template <int NCT, int KS, bool DBF>
__global__ __launch_bounds__(SS_NT, 1) void ss_dgrad_kernel(const void* __restrict__ dy2,
                                                            const uint16_t* __restrict__ y1, float* __restrict__ dy1,
                                                            SdGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sd_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  int cls = 0;
  while (cls < 3 && (int64_t)blockIdx.x >= g.wg0[cls + 1]) ++cls;
  const __amdgpu_buffer_rsrc_t rdy2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)dy2, (short)0, (int)((int64_t)g.B * g.T2 * g.F2 * g.C * (DBF ? 2 : 4)), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)y1, (short)0, (int)((int64_t)g.B * g.T1 * g.F1 * g.ldy * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rdy1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dy1, (short)0, dy1 ? (int)((int64_t)g.B * g.T1 * g.F1 * g.C * 4) : 0, 0x00020000);
  float wacc[NCT][10];
#pragma unroll
  for (int n = 0; n < NCT; ++n)
#pragma unroll
    for (int k = 0; k < 10; ++k) wacc[n][k] = 0.f;
  switch (cls) {
    case 0: sd_class<NCT, KS, 0, 0, DBF>(g, rdy2, ry1, rdy1, dy1 != nullptr, sd_lds, 0, wacc); break;
    case 1: sd_class<NCT, KS, 0, 1, DBF>(g, rdy2, ry1, rdy1, dy1 != nullptr, sd_lds, 1, wacc); break;
    case 2: sd_class<NCT, KS, 1, 0, DBF>(g, rdy2, ry1, rdy1, dy1 != nullptr, sd_lds, 2, wacc); break;
    default: sd_class<NCT, KS, 1, 1, DBF>(g, rdy2, ry1, rdy1, dy1 != nullptr, sd_lds, 3, wacc); break;
  }
  if (!g.wpart) return;
  // per-workgroup partial: lanes r / r + 32 hold the same channels, then the 8 waves in order
#pragma unroll
  for (int n = 0; n < NCT; ++n)
#pragma unroll
    for (int k = 0; k < 10; ++k) wacc[n][k] += __shfl_xor(wacc[n][k], 32, 64);
  __syncthreads();   // the tap slabs and per-wave buffers are no longer read: reuse the LDS
  float* red = reinterpret_cast<float*>(sd_lds);
  if (h == 0) {
#pragma unroll
    for (int n = 0; n < NCT; ++n)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[(wave * NCT * 10 + n * 10 + k) * 32 + r] = wacc[n][k];
  }
  __syncthreads();
  float* wp = g.wpart + (int64_t)blockIdx.x * g.C * 10;
  for (int o = threadIdx.x; o < NCT * 32 * 10; o += SS_NT) {
    const int n = o / 320, rem = o % 320, k = rem / 32, rr = rem % 32;
    const int ci = 32 * n + rr;
    if (ci >= g.C) continue;
    float v = 0.f;
    for (int w = 0; w < SS_WAVES; ++w) v += red[(w * NCT * 10 + n * 10 + k) * 32 + rr];
    if (k < 9) wp[ci * 9 + k] = v;
    else wp[g.C * 9 + ci] = v;
  }
}

// ---- the output Linear's data gradient as the bf16 conv2 output gradient -----------------------------
// dy2h[r][n] = bf16( [y2[r][n] > 0] * sum_k dlin[r][k] W[k][n] ),  n < ncols = F2 * C, k < d <= 32 KS
// (Linear(C F2 -> d) of the channels-last conv2 output, ReLU' of that output): was kdfm_gemm's linear_dx with
// the DRELU epilogue writing f32 (90 MB at the bench shape, 118 us in the step) and a bf16 cast of it for the
// conv2 weight gradient; here one pass writes the bf16 operand that the conv2 data gradient
// (kdfm_subsample_conv2_dgrad_w0_h) and weight gradient both read.  C^T tiles (v_mfma_f32_16x16x32_bf16):
// A = W^T, a slice of SO_TILES x 16 columns staged in LDS from the prepared bf16 [col][k] image
// (kdfm_ss_out_wprep), B = 16 rows of dlin (f32 loads, rounded to bf16 as kdfm_gemm's bf16 math does), so a
// lane ends with 4 consecutive columns of one row: one 16-byte load of y2 for the mask, one 8-byte store.
constexpr int SO_TILES = 11;   // 176 columns per workgroup
constexpr int SO_RT = 4;       // row tiles of 16 per wave (256 rows per workgroup)

__global__ __launch_bounds__(256) void ss_out_wprep_kernel(const float* __restrict__ W, uint16_t* __restrict__ wt, int d,
                                                           int64_t ncols, int KP) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;   // wt[n][k]
  if (idx >= ncols * KP) return;
  const int64_t n = idx / KP;
  const int k = (int)(idx - n * KP);
  wt[idx] = f2bf(k < d ? W[(int64_t)k * ncols + n] : 0.f);
}

template <int KS>
__global__ __launch_bounds__(256) void ss_out_dgrad_kernel(const float* __restrict__ dlin, const uint16_t* __restrict__ wt,
                                                           const float* __restrict__ y2, uint16_t* __restrict__ dy2h,
                                                           int64_t rows, int d, int64_t ncols) {
  constexpr int KP = 32 * KS, LDW = KP + 8, NCOL = SO_TILES * 16, C8 = KP / 8;
  __shared__ __attribute__((aligned(16))) uint16_t Ws[NCOL * LDW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, lo = lane & 15;
  const int64_t n0 = (int64_t)blockIdx.x * NCOL;
  // stage the W^T slice [col][k] (columns past ncols read as zero)
  constexpr int NCH = NCOL * C8, PER = (NCH + 255) / 256;
  bf16x8_t st[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int c = e / C8, k8 = (e - c * C8) * 8;
    st[i] = (e < NCH && n0 + c < ncols) ? *reinterpret_cast<const bf16x8_t*>(wt + (n0 + c) * KP + k8) : bf16x8_t{};
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int c = e / C8, k8 = (e - c * C8) * 8;
    if (e < NCH) *reinterpret_cast<bf16x8_t*>(Ws + c * LDW + k8) = st[i];
  }
  __syncthreads();
  for (int rt = 0; rt < SO_RT; ++rt) {
    const int64_t rb = ((int64_t)blockIdx.y * 4 * SO_RT + w * SO_RT + rt) * 16;
    if (rb >= rows) break;   // wave-uniform
    const int64_t row = rb + lo;
    const bool rin = row < rows;
    // B fragments: dlin[row][32 ks + 8 q .. + 7]
    bf16x8_t bfr[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = 32 * ks + 8 * q;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (rin && c0 + e < d) ? dlin[row * d + c0 + e] : 0.f;
      bfr[ks] = pack_bf16x8<bf16x8_t>(v);
    }
#pragma unroll
    for (int t = 0; t < SO_TILES; ++t) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(Ws + (t * 16 + lo) * LDW + 32 * ks + 8 * q);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[ks], acc, 0, 0, 0);
      }
      // acc[r] = C^T[column n0 + 16 t + 4 q + r][row]
      const int64_t col = n0 + 16 * t + 4 * q;
      if (rin && col < ncols) {
        const float4 m = *reinterpret_cast<const float4*>(y2 + row * ncols + col);
        const float a0 = acc[0], a1 = acc[1], a2 = acc[2], a3 = acc[3];
        const uint2 o = make_uint2(pack_bf16x2(m.x > 0.f ? a0 : 0.f, m.y > 0.f ? a1 : 0.f),
                                   pack_bf16x2(m.z > 0.f ? a2 : 0.f, m.w > 0.f ? a3 : 0.f));
        *reinterpret_cast<uint2*>(dy2h + row * ncols + col) = o;
      }
    }
  }
}

template <int NCT, int KS, bool DBF>
int sd_launch(const void* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, SdGeo g, hipStream_t st) {
  g.wt = wt;
  // 4 tap slabs (the largest class) + per-wave patch / index buffers; the fold reuses the space
  size_t lds = (size_t)4 * 32 * NCT * g.ldb * sizeof(uint16_t) + (size_t)SS_WAVES * (32 * SD_PTS + 32) * 4;
  const size_t red = (size_t)SS_WAVES * NCT * 10 * 32 * sizeof(float);   // fused conv0 wgrad reduction
  if (g.wpart && red > lds) lds = red;
  static bool once = [] {
    (void)hipFuncSetAttribute((const void*)ss_dgrad_kernel<NCT, KS, DBF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    return true;
  }();
  (void)once;
  hipLaunchKernelGGL((ss_dgrad_kernel<NCT, KS, DBF>), dim3((unsigned)g.wg0[4]), dim3(SS_NT), lds, st, dy2, y1, dy1, g);
  return check_launch("kdfm_subsample_conv2_dgrad");
}

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_subsample_wprep_elems(int64_t C) {
  const int64_t Np = kdfm::ceil_div(C, 32) * 32, Cp = kdfm::ceil_div(C, 16) * 16;
  return Np * 9 * Cp;
}

int kdfm_subsample_wprep(const float* w2, uint16_t* wb, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(w2 && wb && C > 0, "bad arguments");
  const int64_t Np = ceil_div(C, 32) * 32, Cp = ceil_div(C, 16) * 16;
  const int64_t n = Np * 9 * Cp;
  hipLaunchKernelGGL(ss_wprep_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), w2, wb,
                     (int)C, (int)Np, (int)Cp);
  return check_launch("kdfm_subsample_wprep");
}

int kdfm_subsample_conv1(const float* mel, const int64_t* mel_len, const int64_t* len1, const float* w0,
                         const float* b0, uint16_t* y1b, float* y1f, int64_t B, int64_t Tm, int64_t F, int64_t C,
                         void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(mel && w0 && b0 && y1b, "null pointer");
  KDFM_REQUIRE(C % 8 == 0 && B > 0 && Tm > 0 && F > 0, "C must be a multiple of 8");
  const int64_t T1 = (Tm - 1) / 2 + 1, F1 = (F - 1) / 2 + 1;
  const int64_t n = B * T1 * F1 * (C / 8);
  KDFM_REQUIRE(n < (1ll << 31) && C <= 256, "too large (32-bit indexing, C <= 256)");
  hipLaunchKernelGGL(ss_conv1_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), mel, mel_len,
                     len1, w0, b0, y1b, y1f, (int)B, (int)Tm, (int)F, (int)C, (int)T1, (int)F1);
  return check_launch("kdfm_subsample_conv1");
}

int kdfm_subsample_conv2(const uint16_t* y1b, const int64_t* len2, const uint16_t* wb, const float* b2, float* y2,
                         int64_t B, int64_t T1, int64_t F1, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(y1b && wb && b2 && y2, "null pointer");
  KDFM_REQUIRE(C % 8 == 0 && C <= 192 && B > 0 && T1 > 0 && F1 > 0, "C must be a multiple of 8, <= 192");
  KDFM_REQUIRE((((uintptr_t)y1b) & 15) == 0 && (((uintptr_t)wb) & 15) == 0, "y1b / wb must be 16-byte aligned");
  SsGeo g;
  g.B = (int)B; g.T1 = (int)T1; g.F1 = (int)F1; g.C = (int)C;
  g.T2 = (int)((T1 - 1) / 2 + 1); g.F2 = (int)((F1 - 1) / 2 + 1);
  g.P = B * g.T2 * g.F2;
  g.Cp = (int)(ceil_div(C, 16) * 16);
  g.ldb = g.Cp + 8;
  const int nct = (int)ceil_div(C, 32), ks = g.Cp / 16;
  hipStream_t st = as_stream(stream);
  if (nct == 3 && ks == 6) return ss_launch<3, 1, 6>(y1b, len2, wb, b2, y2, g, st);    // d = 88 / 96
  if (nct == 6 && ks == 11) return ss_launch<3, 2, 11>(y1b, len2, wb, b2, y2, g, st);  // d = 176
  if (nct == 6 && ks == 12) return ss_launch<3, 2, 12>(y1b, len2, wb, b2, y2, g, st);  // d = 192
  if (nct == 1 && ks == 2) return ss_launch<1, 1, 2>(y1b, len2, wb, b2, y2, g, st);    // tiny test sizes
  if (nct == 2 && ks == 4) return ss_launch<1, 2, 4>(y1b, len2, wb, b2, y2, g, st);
  set_error("kdfm_subsample_conv2: unsupported channel count");
  return KDFM_EUNSUPPORTED;
}

int64_t kdfm_subsample_dgrad_wprep_elems(int64_t C) {
  return 9 * kdfm::ceil_div(C, 32) * 32 * kdfm::ceil_div(C, 16) * 16;
}

int kdfm_subsample_dgrad_wprep(const float* w2, uint16_t* wt, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(w2 && wt && C > 0, "bad arguments");
  const int64_t Np = ceil_div(C, 32) * 32, Cp = ceil_div(C, 16) * 16;
  const int64_t n = 9 * Np * Cp;
  hipLaunchKernelGGL(ss_dgrad_wprep_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), w2, wt,
                     (int)C, (int)Np, (int)Cp);
  return check_launch("kdfm_subsample_dgrad_wprep");
}

}  // extern "C"

namespace kdfm {
namespace {
int sd_geo(SdGeo& g, int64_t B, int64_t T1, int64_t F1, int64_t C) {
  g.B = (int)B; g.T1 = (int)T1; g.F1 = (int)F1; g.C = (int)C;
  g.ldy = (int)C;
  g.T2 = (int)((T1 - 1) / 2 + 1); g.F2 = (int)((F1 - 1) / 2 + 1);
  g.Cp = (int)(ceil_div(C, 16) * 16);
  g.ldb = g.Cp + 8;
  g.wg0[0] = 0;
  for (int c = 0; c < 4; ++c) {
    const int pt = c >> 1, pf = c & 1;
    g.npos[c] = B * ((T1 - pt + 1) / 2) * ((F1 - pf + 1) / 2);
    g.wg0[c + 1] = g.wg0[c] + ceil_div(ceil_div(g.npos[c], 32 * SS_WAVES), SD_TPW);
  }
  g.mel = nullptr; g.mel_len = nullptr; g.Tm = g.Fm = g.pad = 0; g.wpart = nullptr; g.wt = nullptr;
  return 0;
}
template <bool DBF>
int sd_dispatch(const void* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, const SdGeo& g, hipStream_t st) {
  const int nct = (int)ceil_div(g.C, 32), ks = g.Cp / 16;
  if (nct == 3 && ks == 6) return sd_launch<3, 6, DBF>(dy2, wt, y1, dy1, g, st);    // d = 88 / 96
  if (nct == 1 && ks == 1) return sd_launch<1, 1, DBF>(dy2, wt, y1, dy1, g, st);    // test sizes
  if (nct == 1 && ks == 2) return sd_launch<1, 2, DBF>(dy2, wt, y1, dy1, g, st);
  if (nct == 2 && ks == 4) return sd_launch<2, 4, DBF>(dy2, wt, y1, dy1, g, st);
  set_error("kdfm_subsample_conv2_dgrad: unsupported channel count");
  return KDFM_EUNSUPPORTED;
}
}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_subsample_conv2_dgrad_w0_ws(int64_t B, int64_t T1, int64_t F1, int64_t C) {
  kdfm::SdGeo g;
  kdfm::sd_geo(g, B, T1, F1, C);
  return g.wg0[4] * C * 10;
}

}  // extern "C"

namespace kdfm {
namespace {
template <bool DBF>
int sd_w0(const void* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B, int64_t T1, int64_t F1,
          int64_t C, int64_t ldy1, const float* mel, const int64_t* mel_len, int64_t Tm, int64_t Fm, int64_t pad, float* dw0,
          float* db0, float* ws, int64_t ws_len, void* stream) {
  KDFM_REQUIRE(dy2 && wt && y1 && mel && dw0 && db0 && ws, "null pointer");
  KDFM_REQUIRE(C % 8 == 0 && B > 0 && T1 > 0 && F1 > 0, "C must be a multiple of 8");
  KDFM_REQUIRE(((((uintptr_t)dy2) | ((uintptr_t)wt)) & 15) == 0, "dy2 / wt must be 16-byte aligned");
  KDFM_REQUIRE(T1 == (Tm + 2 * pad - 3) / 2 + 1 && F1 == (Fm + 2 * pad - 3) / 2 + 1, "conv0 geometry");
  KDFM_REQUIRE(ldy1 >= C, "ldy1 < C");
  SdGeo g;
  sd_geo(g, B, T1, F1, C);
  g.ldy = (int)ldy1;
  KDFM_REQUIRE(g.wg0[4] < (1ll << 31) && B * T1 * F1 * C * 4 < (1ll << 31) && B * T1 * F1 * ldy1 * 2 < (1ll << 31) &&
               B * Tm * Fm < (1ll << 31),
               "too large (32-bit buffer offsets: dy1 / y1 / dy2 < 2 GiB)");
  KDFM_REQUIRE(ws_len >= g.wg0[4] * C * 10, "workspace too small (kdfm_subsample_conv2_dgrad_w0_ws)");
  g.mel = mel; g.mel_len = mel_len; g.Tm = (int)Tm; g.Fm = (int)Fm; g.pad = (int)pad; g.wpart = ws;
  hipStream_t st = as_stream(stream);
  int rc = sd_dispatch<DBF>(dy2, wt, y1, dy1, g, st);
  if (rc) return rc;
  // fixed-order fold of the per-workgroup partials: dW0 (C, 9) += sum_wg, db0 (C) += sum_wg
  return launch_colsum2(ws, dw0, C * 9, db0, g.wg0[4], C * 10, C * 10, 1.f, st);
}
}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_subsample_conv2_dgrad_w0(const float* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B,
                                  int64_t T1, int64_t F1, int64_t C, int64_t ldy1, const float* mel, const int64_t* mel_len,
                                  int64_t Tm, int64_t Fm, int64_t pad, float* dw0, float* db0, float* ws,
                                  int64_t ws_len, void* stream) {
  return kdfm::sd_w0<false>(dy2, wt, y1, dy1, B, T1, F1, C, ldy1, mel, mel_len, Tm, Fm, pad, dw0, db0, ws, ws_len, stream);
}

int kdfm_subsample_conv2_dgrad_w0_h(const uint16_t* dy2h, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B,
                                    int64_t T1, int64_t F1, int64_t C, int64_t ldy1, const float* mel, const int64_t* mel_len,
                                    int64_t Tm, int64_t Fm, int64_t pad, float* dw0, float* db0, float* ws,
                                    int64_t ws_len, void* stream) {
  return kdfm::sd_w0<true>(dy2h, wt, y1, dy1, B, T1, F1, C, ldy1, mel, mel_len, Tm, Fm, pad, dw0, db0, ws, ws_len, stream);
}

int kdfm_subsample_conv2_dgrad(const float* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B, int64_t T1,
                               int64_t F1, int64_t C, int64_t ldy1, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dy2 && wt && y1 && dy1, "null pointer");
  KDFM_REQUIRE(C % 8 == 0 && B > 0 && T1 > 0 && F1 > 0, "C must be a multiple of 8");
  KDFM_REQUIRE(ldy1 >= C, "ldy1 < C");
  KDFM_REQUIRE(((((uintptr_t)dy2) | ((uintptr_t)wt)) & 15) == 0, "dy2 / wt must be 16-byte aligned");
  SdGeo g;
  sd_geo(g, B, T1, F1, C);
  g.ldy = (int)ldy1;
  KDFM_REQUIRE(g.wg0[4] < (1ll << 31) && B * T1 * F1 * C * 4 < (1ll << 31) && B * T1 * F1 * ldy1 * 2 < (1ll << 31),
               "too large (32-bit buffer offsets: dy1 / y1 / dy2 < 2 GiB)");
  return sd_dispatch<false>(dy2, wt, y1, dy1, g, as_stream(stream));
}

int64_t kdfm_ss_out_wprep_elems(int64_t d, int64_t ncols) {
  if (d <= 0 || d > 128 || ncols <= 0) return -1;
  return ncols * 32 * kdfm::ceil_div(d, 32);
}

int kdfm_ss_out_wprep(const float* W, uint16_t* wt, int64_t d, int64_t ncols, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(W && wt, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 128 && ncols > 0, "d must be in (0, 128]");
  const int KP = (int)(32 * ceil_div(d, 32));
  const int64_t n = ncols * KP;
  hipLaunchKernelGGL(ss_out_wprep_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), W, wt,
                     (int)d, ncols, KP);
  return check_launch("kdfm_ss_out_wprep");
}

int kdfm_ss_out_dgrad(const float* dlin, const uint16_t* wt, const float* y2, uint16_t* dy2h, int64_t rows, int64_t d,
                      int64_t ncols, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dlin && wt && y2 && dy2h, "null pointer");
  KDFM_REQUIRE(d > 0 && d <= 128 && ncols > 0 && ncols % 4 == 0, "d in (0, 128], ncols a multiple of 4");
  KDFM_REQUIRE((((uintptr_t)wt | (uintptr_t)y2) & 15) == 0 && ((uintptr_t)dy2h & 7) == 0, "operands misaligned");
  if (rows == 0) return KDFM_OK;
  const dim3 grid((unsigned)ceil_div(ncols, SO_TILES * 16), (unsigned)ceil_div(rows, 64 * SO_RT));
  hipStream_t st = as_stream(stream);
  const int ks = (int)ceil_div(d, 32);
  if (ks == 1) hipLaunchKernelGGL(ss_out_dgrad_kernel<1>, grid, dim3(256), 0, st, dlin, wt, y2, dy2h, rows, (int)d, ncols);
  else if (ks == 2) hipLaunchKernelGGL(ss_out_dgrad_kernel<2>, grid, dim3(256), 0, st, dlin, wt, y2, dy2h, rows, (int)d, ncols);
  else if (ks == 3) hipLaunchKernelGGL(ss_out_dgrad_kernel<3>, grid, dim3(256), 0, st, dlin, wt, y2, dy2h, rows, (int)d, ncols);
  else hipLaunchKernelGGL(ss_out_dgrad_kernel<4>, grid, dim3(256), 0, st, dlin, wt, y2, dy2h, rows, (int)d, ncols);
  return check_launch("kdfm_ss_out_dgrad");
}

}  // extern "C"
