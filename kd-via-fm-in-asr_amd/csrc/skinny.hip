// Weight-stationary skinny GEMM for the Conformer / KD-head products (bf16 MFMA 32x32x16, f32
// accumulate):  C[M x N] = epi(alpha * A[M x K] * B[K x N]),  M >> N, K (N, K <= a few hundred).
//
// Every Linear / 1x1 conv / k=3 time conv of the ver5 step and its data-gradient has this shape:
// 12,832 rows (B*T' frames) for the encoders (conformer_encoder.py:685-692, App. A.5-A.8) and
// 205,312 rows (16 layers x B*T') for the stacked KD heads (asr_train_diffm.py:400-497), against
// 88..704 output channels.  Such a product is HBM/latency bound, so the kernel is shaped around
// streaming the activation exactly once with many bytes in flight:
//
//  * a workgroup owns a column range of B (weights) and stages it ONCE, as bf16, into LDS
//    ([n][k] image, k padded to 16); it then walks row tiles persistently (grid-stride), so the
//    weight staging is amortised over all the rows it processes;
//  * each wave computes a 32-row x (32*NCT)-column tile with v_mfma_f32_32x32x16_bf16; its A
//    fragments are loaded straight from HBM into registers (8 consecutive k per lane, f32 ->
//    bf16 in registers; no LDS, no barrier in the row loop) in chunks of 96 k, and the next
//    chunk/tile is prefetched while the MFMAs of the current one run;
//  * CONV mode (Conv1d k=3 along frames, per-utterance zero padding): chunk c = tap c reads the
//    shifted rows m + c - pad, so the conv never materialises an im2col matrix;
//  * the fused epilogue is the shared per-element epilogue_store (bias, ReLU/SiLU, STORE_PRE,
//    counter-RNG dropout, dReLU/dSiLU, residual, beta, row mask, MSE) — identical semantics to
//    the generic kernel; the 32x32 accumulator layout stores 128 contiguous bytes per half-wave.
//
// Selected inside kdfm_gemm for bf16 math (the f32 parity mode keeps the generic kernel), so the
// C-ABI and every call site are unchanged.
#include "gemm_common.h"

#include <cstdlib>

namespace kdfm {
namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int SK_CKS = 6;             // k-steps (16 k each) per A chunk in KC mode
constexpr int SK_CHUNK = 16 * SK_CKS; // 96
constexpr int SK_EPS = 36;            // f32 row stride of the per-wave epilogue tile (16-B rows)

// wave-local LDS hand-off: this wave's ds_writes complete before its following ds_reads
__device__ __forceinline__ void sk_wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

struct SkGeo {
  int Kp;       // B image k extent (K rounded up to 16)
  int ldb;      // B image row stride in bf16 elements (Kp + 8)
  int chunk;    // k per A chunk (96 in KC mode, conv_c in CONV mode); multiple of 16
  int nchunks;  // chunks per row tile
  int cw;       // columns per column range (= 32 * NCT * gcols)
  int gcols;    // waves sharing one row tile (column groups)
  int64_t tiles;  // 32-row tiles
};

__device__ __forceinline__ void pk4(uint16_t* dst, float4 v) {
  const uint32_t lo = pack_bf16x2(v.x, v.y);
  const uint32_t hi = pack_bf16x2(v.z, v.w);
  *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
}

__device__ __forceinline__ bf16x8 cvt8(float4 a, float4 b) {
  const float t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return pack_bf16x8<bf16x8>(t);
}

// Stage B columns [n0, n0 + cw) x k [0, Kp) into the bf16 [n][k] image (zero outside N / K).
// Predicated loads as UNCONDITIONAL loads from a clamped address + a select.  Written as
// `ok ? *ptr : 0` the compiler branches around each load and waits vmcnt(0) inside the branch,
// serialising a batch of loads into one memory latency each (the weight staging took ~13 us per
// launch that way).  `base` must be a valid address (the operand's first element).
__device__ __forceinline__ float4 ld4_or0(const float* base, int64_t off, bool ok) {
  const float4 t = *reinterpret_cast<const float4*>(base + (ok ? off : 0));
  return ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ float ld_or0(const float* base, int64_t off, bool ok) {
  const float t = base[ok ? off : 0];
  return ok ? t : 0.f;
}

__device__ void sk_stage_B(const GemmP& p, const SkGeo& g, uint16_t* Bs, int64_t n0) {
  const int nth = blockDim.x, tid = threadIdx.x;
  const int cw = g.cw, Kp = g.Kp, ldb = g.ldb;
  if (p.sBk == 1 && (p.K & 3) == 0 && (p.sBn & 3) == 0 && ((((uintptr_t)p.B) & 15) == 0)) {
    // W[n][k]: float4 along k
    const int kq = Kp >> 2;
    const int total = cw * kq;
    for (int base = 0; base < total; base += nth * 4) {
      float4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + tid + i * nth;
        const int nl = e / kq, k = (e - nl * kq) * 4;
        const int64_t n = n0 + nl;
        v[i] = ld4_or0(p.B, n * p.sBn + k, e < total && n < p.N && k < p.K);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + tid + i * nth;
        if (e < total) {
          const int nl = e / kq, k = (e - nl * kq) * 4;
          pk4(Bs + nl * ldb + k, v[i]);
        }
      }
    }
  } else if (p.sBn == 1 && (p.N & 3) == 0 && (p.sBk & 3) == 0 && ((((uintptr_t)p.B) & 15) == 0) &&
             (n0 & 3) == 0) {
    // B(k, n) contiguous along n: float4 along n, transposed into the image
    const int nq = cw >> 2;
    const int total = Kp * nq;
    for (int base = 0; base < total; base += nth * 4) {
      float4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + tid + i * nth;
        const int k = e / nq, nl = (e - k * nq) * 4;
        const int64_t n = n0 + nl;
        v[i] = ld4_or0(p.B, (int64_t)k * p.sBk + n, e < total && n < p.N && k < p.K);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = base + tid + i * nth;
        if (e < total) {
          const int k = e / nq, nl = (e - k * nq) * 4;
          Bs[(nl + 0) * ldb + k] = f2bf(v[i].x);
          Bs[(nl + 1) * ldb + k] = f2bf(v[i].y);
          Bs[(nl + 2) * ldb + k] = f2bf(v[i].z);
          Bs[(nl + 3) * ldb + k] = f2bf(v[i].w);
        }
      }
    }
  } else {
    for (int e = tid; e < cw * Kp; e += nth) {
      const int nl = e / Kp, k = e - nl * Kp;
      const int64_t n = n0 + nl;
      const float x = ld_or0(p.B, (int64_t)k * p.sBk + n * p.sBn, n < p.N && k < p.K);
      Bs[nl * ldb + k] = f2bf(x);
    }
  }
}

// A chunk for one wave: lane (r = lane&31, h = lane>>5) holds, for k-step s, the 8 values
// A(m0 + r, kc + 16 s + 8 h + j), j = 0..7 (two float4 loads); zero outside M / K / utterance.
template <int AMODE>
__device__ __forceinline__ void sk_load_A(float4 (&v)[SK_CKS][2], const GemmP& p, const SkGeo& g, int64_t m0,
                                          int c, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int64_t m = m0 + r;
  int64_t row = m;
  bool ok = m < p.M;
  int kbase;
  if constexpr (AMODE == KDFM_LD_CONV) {
    // chunk c is tap c: rows shifted by c - pad, zero outside the utterance
    const int64_t t = m % p.conv_t;
    const int64_t tt = t + c - p.pad;
    ok = ok && tt >= 0 && tt < p.conv_t;
    row = m + c - p.pad;
    kbase = 0;
  } else {
    kbase = c * SK_CHUNK;
  }
  const int klim = (AMODE == KDFM_LD_CONV) ? (int)p.conv_c : (int)p.K;
#pragma unroll
  for (int s = 0; s < SK_CKS; ++s) {
    const int k = kbase + 16 * s + 8 * h;
    if (16 * s < g.chunk) {  // compile-time after unrolling for the common chunk sizes
      const bool okk = ok && k < klim;
      const int64_t off = (row * p.sAm + k) * (okk ? 1 : 0);
      v[s][0] = ld4_or0(p.A, off, okk);
      v[s][1] = ld4_or0(p.A, off + 4, okk);
    } else {
      v[s][0] = make_float4(0.f, 0.f, 0.f, 0.f);
      v[s][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// (compile-time epilogues SKC_EPI_*: gemm_common.h)
template <int NCT, int AMODE, int WV, int EMODE = SKC_EPI_GENERIC>
__global__ __launch_bounds__(64 * WV, 2) void sk_fwd_kernel(GemmP p, SkGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sk_lds[];
  uint16_t* Bs = sk_lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ncr0 = (int64_t)blockIdx.y * g.cw;
  sk_stage_B(p, g, Bs, ncr0);
  __syncthreads();

  const int cg = wave % g.gcols;
  const int rpi = WV / g.gcols;                 // row tiles per workgroup iteration
  const int rsub = wave / g.gcols;
  if (rsub >= rpi) return;                      // (WV not a multiple of gcols)
  const int nl0 = cg * 32 * NCT;                // first image column of this wave
  const int64_t n0 = ncr0 + nl0;
  if (n0 >= p.N) return;                        // no columns for this wave (no barrier follows)
  const int r = lane & 31, h = lane >> 5;
  const int64_t tstride = (int64_t)gridDim.x * rpi;
  const int64_t tfirst = (int64_t)blockIdx.x * rpi + rsub;
  if (tfirst >= g.tiles) return;
  const int64_t ntile = (g.tiles - tfirst + tstride - 1) / tstride;
  const int64_t nsteps = ntile * g.nchunks;

  const int epi = p.epi;
  const uint64_t seed = (epi & KDFM_EPI_DROPOUT) ? load_seed(p.seed) : 0ull;
  const float keep_scale = (epi & KDFM_EPI_DROPOUT) ? 1.f / (1.f - p.dropout_p) : 1.f;
  bool single;
  const float* side = epi_side_src(p, single);  // the dispatcher guarantees `single`
  float mse_part = 0.f;
  // Epilogue lane map (row-major, 16-byte global accesses): the 32x32 accumulator tile is turned
  // around through a per-wave LDS tile, then lane -> rows er + 8 i (i < 4), columns ec..ec+3 of each
  // 32-column tile j.  Scalar 4-byte stores issue-limit the write stream (MI355X_MICROARCH.md,
  // 'epilogue store tail'); dwordx4 stores and loads move 4x the bytes per instruction.
  const int er = lane >> 3, ec = (lane & 7) * 4;
  float* Ep = reinterpret_cast<float*>(sk_lds + (size_t)g.cw * g.ldb) + wave * 32 * SK_EPS;
  float4 bn4[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) {
    float t[4];
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int64_t n = n0 + 32 * j + ec + c4;
      t[c4] = ((epi & KDFM_EPI_BIAS) && n < p.N) ? p.bias[n] : 0.f;
    }
    bn4[j] = make_float4(t[0], t[1], t[2], t[3]);
  }

  const uint16_t* bp = Bs + (nl0 + r) * g.ldb + 8 * h;
  f32x16 acc[NCT];
  float4 av[SK_CKS][2];
  sk_load_A<AMODE>(av, p, g, tfirst * 32, 0, lane);
  int c = 0;
  int64_t tile = tfirst;
  for (int64_t q = 0; q < nsteps; ++q) {
    const bool last = (c == g.nchunks - 1);
    const int64_t m0 = tile * 32;
    // side operands of this tile's epilogue (row-major float4): issued before the prefetch and MFMAs
    float4 sv4[NCT][4];
    bool rowok[4];
    if (last) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = m0 + er + 8 * i;
        rowok[i] = m < p.M && epi_row_ok(p, m < p.M ? m : 0);
      }
      if (side) {
#pragma unroll
        for (int j = 0; j < NCT; ++j) {
          const int64_t n = n0 + 32 * j + ec;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int64_t m = m0 + er + 8 * i;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n + 3 < p.N) {
              v = ld4_or0(side, m * p.sCm + n, m < p.M);
            } else if (m < p.M && n < p.N) {
              v.x = side[m * p.sCm + n];
              if (n + 1 < p.N) v.y = side[m * p.sCm + n + 1];
              if (n + 2 < p.N) v.z = side[m * p.sCm + n + 2];
            }
            sv4[j][i] = v;
          }
        }
      }
    }
    bf16x8 af[SK_CKS];
#pragma unroll
    for (int s = 0; s < SK_CKS; ++s) af[s] = cvt8(av[s][0], av[s][1]);
    // prefetch the next (tile, chunk)
    {
      int c2 = c + 1;
      int64_t t2 = tile;
      if (c2 == g.nchunks) { c2 = 0; t2 += tstride; }
      if (q + 1 < nsteps) sk_load_A<AMODE>(av, p, g, t2 * 32, c2, lane);
    }
    if (c == 0) {
#pragma unroll
      for (int j = 0; j < NCT; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
    }
    const int kimg = c * g.chunk;
#pragma unroll
    for (int s = 0; s < SK_CKS; ++s) {
      if (16 * s < g.chunk) {
#pragma unroll
        for (int j = 0; j < NCT; ++j) {
          const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(bp + j * 32 * g.ldb + kimg + 16 * s);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bfr, acc[j], 0, 0, 0);
        }
      }
    }
    if (last) {
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
#pragma unroll
        for (int i = 0; i < 16; ++i) Ep[((i & 3) + 8 * (i >> 2) + 4 * h) * SK_EPS + r] = acc[j][i];
        sk_wave_lds_sync();
        const int64_t n = n0 + 32 * j + ec;
        const float bv[4] = {bn4[j].x, bn4[j].y, bn4[j].z, bn4[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = er + 8 * i;
          const int64_t m = m0 + row;
          const float4 a = *reinterpret_cast<const float4*>(Ep + row * SK_EPS + ec);
          if (m >= p.M || n >= p.N) continue;
          const float av4[4] = {a.x, a.y, a.z, a.w};
          const float s4[4] = {sv4[j][i].x, sv4[j][i].y, sv4[j][i].z, sv4[j][i].w};
          float o[4], pr[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = 0.f;
            pr[e] = 0.f;
            if (n + e < p.N)
              o[e] = skc_epi<EMODE>(p, m, n + e, p.alpha * av4[e], bv[e], side ? s4[e] : 0.f, rowok[i], seed,
                                    keep_scale, mse_part, pr[e]);
          }
          const int64_t off = m * p.sCm + n;
          if (n + 3 < p.N) {
            *reinterpret_cast<float4*>(p.C + off) = make_float4(o[0], o[1], o[2], o[3]);
            if (epi & KDFM_EPI_STORE_PRE)
              *reinterpret_cast<float4*>(p.Cpre + off) = make_float4(pr[0], pr[1], pr[2], pr[3]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < p.N) {
                p.C[off + e] = o[e];
                if (epi & KDFM_EPI_STORE_PRE) p.Cpre[off + e] = pr[e];
              }
          }
        }
        sk_wave_lds_sync();  // Ep is rewritten for the next column tile
      }
      c = 0;
      tile += tstride;
    } else {
      ++c;
    }
  }
  if (epi & KDFM_EPI_MSE) {
    mse_part = wave_sum(mse_part);
    if (lane == 0) atomicAdd(p.loss_acc, mse_part * p.loss_scale);
  }
}

// Direct-B variant (p.Bh set): no LDS at all.  Work items are (32-row tile, column group) pairs
// spread over every wave of the grid; B fragments are 16-byte loads from the bf16 weight twin
// (L2-resident), issued together with the A loads, so a K <= 96 product is one memory round trip
// per wave plus the epilogue.  Waves of one workgroup take the column groups of the same row tile,
// so the repeated A rows hit L1/L2.
template <int NCT, int AMODE>
__global__ __launch_bounds__(256, 2) void skd_fwd_kernel(GemmP p, SkGeo g, int G) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t wglob = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t wstride = (int64_t)gridDim.x * 4;
  const int64_t ntasks = g.tiles * G;
  if (wglob >= ntasks) return;
  const int64_t nmine = (ntasks - wglob + wstride - 1) / wstride;
  const int64_t nsteps = nmine * g.nchunks;

  const int epi = p.epi;
  const uint64_t seed = (epi & KDFM_EPI_DROPOUT) ? load_seed(p.seed) : 0ull;
  const float keep_scale = (epi & KDFM_EPI_DROPOUT) ? 1.f / (1.f - p.dropout_p) : 1.f;
  bool single;
  const float* side = epi_side_src(p, single);
  float mse_part = 0.f;

  f32x16 acc[NCT];
  float4 av[SK_CKS][2];
  int64_t task = wglob;
  sk_load_A<AMODE>(av, p, g, (task / G) * 32, 0, lane);
  int c = 0;
  for (int64_t q = 0; q < nsteps; ++q) {
    const bool last = (c == g.nchunks - 1);
    const int64_t m0 = (task / G) * 32;
    const int64_t n0 = (int64_t)(task % G) * 32 * NCT;
    const int kimg = c * g.chunk;
    // B fragments of this chunk (bf16 twin, row n contiguous along k)
    bf16x8 bfr[SK_CKS][NCT];
#pragma unroll
    for (int s = 0; s < SK_CKS; ++s)
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
        const int64_t n = n0 + 32 * j + r;
        const int k = kimg + 16 * s + 8 * h;
        if (16 * s < g.chunk && n < p.N && k < p.K)
          bfr[s][j] = *reinterpret_cast<const bf16x8*>(p.Bh + n * p.sBh + k);
        else
          bfr[s][j] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    bf16x8 af[SK_CKS];
#pragma unroll
    for (int s = 0; s < SK_CKS; ++s) af[s] = cvt8(av[s][0], av[s][1]);
    {
      int c2 = c + 1;
      int64_t t2 = task;
      if (c2 == g.nchunks) { c2 = 0; t2 += wstride; }
      if (q + 1 < nsteps) sk_load_A<AMODE>(av, p, g, (t2 / G) * 32, c2, lane);
    }
    if (c == 0) {
#pragma unroll
      for (int j = 0; j < NCT; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < SK_CKS; ++s)
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bfr[s][j], acc[j], 0, 0, 0);
    if (last) {
      // side operands after the MFMAs: their latency overlaps the A prefetch already in flight
      float sv[NCT][16], bn[NCT];
      bool rowok[16];
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
        const int64_t n = n0 + 32 * j + r;
        bn[j] = ((epi & KDFM_EPI_BIAS) && n < p.N) ? p.bias[n] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t m = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
        rowok[i] = m < p.M && epi_row_ok(p, m < p.M ? m : 0);
      }
      if (side) {
#pragma unroll
        for (int j = 0; j < NCT; ++j) {
          const int64_t n = n0 + 32 * j + r;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int64_t m = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            sv[j][i] = ld_or0(side, m * p.sCm + n * p.sCn, m < p.M && n < p.N);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
        const int64_t n = n0 + 32 * j + r;
        const bool nok = n < p.N;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int64_t m = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (!nok || m >= p.M) continue;
          float pre = 0.f;
          const float v = epi_apply(p, 0, m, n, p.alpha * acc[j][i], bn[j], side ? sv[j][i] : 0.f, rowok[i], seed,
                                    keep_scale, mse_part, pre);
          const int64_t off = m * p.sCm + n * p.sCn;
          if (epi & KDFM_EPI_STORE_PRE) p.Cpre[off] = pre;
          p.C[off] = v;
        }
      }
      c = 0;
      task += wstride;
    } else {
      ++c;
    }
  }
  if (epi & KDFM_EPI_MSE) {
    mse_part = wave_sum(mse_part);
    if (lane == 0) atomicAdd(p.loss_acc, mse_part * p.loss_scale);
  }
}

// ------------------------------------------------------------------------------------------------
// CONV mode with an LDS slab (the denoiser k=3 convolutions, asr_train_diffm.py:444-460, stacked
// over 16 layers: 205,312 rows x 96 channels).  The register-fragment loader above reads each row
// three times (once per tap, 32 B per lane across 32 rows: 32 cache lines per instruction) and
// PMC shows ~1.25x the algorithmic bytes.  Here a wave loads its tile's rows m0-pad .. m0+31+taps-1-pad
// ONCE, as contiguous float4 (1 KiB per instruction, every line fully used), converts them to bf16
// into a per-wave LDS slab, and the three taps read their A fragments from that slab at row
// offsets r + tap (per-lane zero select where the tap crosses an utterance boundary).  The next
// tile's slab is prefetched into registers while the MFMAs and the epilogue of the current one run.
// 8 waves share one staged weight image (96 x 288 bf16); the epilogue's transposition tile aliases
// the wave's slab (free once the MFMAs have read it).
#ifndef KDFM_SKC_WV
#define KDFM_SKC_WV 8  // waves per workgroup (one workgroup per CU: the staged weight image is shared)
#endif
constexpr int SKC_WV = KDFM_SKC_WV;
constexpr int SKC_SLAB_V = 13;            // float4 per lane: (32 + 2) rows x 96 ch / 4 / 64 lanes
constexpr int SKC_LDA = SK_CHUNK + 8;     // bf16 slab row stride (208 B, 16-B aligned)
constexpr int SKC_SLAB_BYTES = 34 * SKC_LDA * 2;

__device__ __forceinline__ void skc_load_slab(float4 (&v)[SKC_SLAB_V], const GemmP& p, int64_t m0, int rows, int cq,
                                              int lane) {
  const int total = rows * cq;
#pragma unroll
  for (int i = 0; i < SKC_SLAB_V; ++i) {
    const int e = lane + 64 * i;
    const int j = e / cq, q = e - j * cq;
    const int64_t gr = m0 - p.pad + j;
    v[i] = ld4_or0(p.A, gr * p.sAm + 4 * q, e < total && gr >= 0 && gr < p.M);
  }
}

template <int NCT, int EMODE>
__global__ __launch_bounds__(64 * SKC_WV, 1) void skc_fwd_kernel(GemmP p, SkGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sk_lds[];
  uint16_t* Bs = sk_lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  sk_stage_B(p, g, Bs, 0);
  __syncthreads();

  const int r = lane & 31, h = lane >> 5;
  const int64_t tstride = (int64_t)gridDim.x * SKC_WV;
  int64_t tile = (int64_t)blockIdx.x * SKC_WV + wave;
  if (tile >= g.tiles) return;
  const int C = (int)p.conv_c, cq = C >> 2, taps = p.taps;
  const int rows = 32 + taps - 1;
  const int64_t T = p.conv_t;

  uint16_t* As = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(sk_lds) + (size_t)g.cw * g.ldb * 2 +
                                             (size_t)wave * SKC_SLAB_BYTES);
  float* Ep = reinterpret_cast<float*>(As);  // epilogue tile (32 x SK_EPS f32) aliases the slab

  const int epi = p.epi;
  const uint64_t seed = (epi & KDFM_EPI_DROPOUT) ? load_seed(p.seed) : 0ull;
  const float keep_scale = (epi & KDFM_EPI_DROPOUT) ? 1.f / (1.f - p.dropout_p) : 1.f;
  bool single;
  const float* side = epi_side_src(p, single);
  float mse_part = 0.f;
  const int er = lane >> 3, ec = (lane & 7) * 4;
  float4 bn4[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) {
    float t4[4];
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) {
      const int64_t n = 32 * j + ec + c4;
      t4[c4] = ((epi & KDFM_EPI_BIAS) && n < p.N) ? p.bias[n] : 0.f;
    }
    bn4[j] = make_float4(t4[0], t4[1], t4[2], t4[3]);
  }
  const uint16_t* bp = Bs + r * g.ldb + 8 * h;

  float4 sv[SKC_SLAB_V];
  skc_load_slab(sv, p, tile * 32, rows, cq, lane);
  for (; tile < g.tiles; tile += tstride) {
    const int64_t m0 = tile * 32;
    // slab registers -> bf16 LDS slab
#pragma unroll
    for (int i = 0; i < SKC_SLAB_V; ++i) {
      const int e = lane + 64 * i;
      if (e < rows * cq) {
        const int j = e / cq, q = e - j * cq;
        pk4(As + j * SKC_LDA + 4 * q, sv[i]);
      }
    }
    sk_wave_lds_sync();
    // next slab prefetch: its latency overlaps the MFMAs and the epilogue of this tile
    if (tile + tstride < g.tiles) skc_load_slab(sv, p, (tile + tstride) * 32, rows, cq, lane);

    f32x16 acc[NCT];
#pragma unroll
    for (int j = 0; j < NCT; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
    const int64_t m = m0 + r;
    const int64_t t = m % T;
    for (int c = 0; c < taps; ++c) {
      const int64_t tt = t + c - p.pad;
      const bool ok = m < p.M && tt >= 0 && tt < T;
      const uint16_t* ap = As + (r + c) * SKC_LDA + 8 * h;
#pragma unroll
      for (int s = 0; s < SK_CKS; ++s) {
        if (16 * s < C) {
          bf16x8 af = *reinterpret_cast<const bf16x8*>(ap + 16 * s);
          if (!ok) af = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
          for (int j = 0; j < NCT; ++j) {
            const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(bp + j * 32 * g.ldb + c * C + 16 * s);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[j], 0, 0, 0);
          }
        }
      }
    }
    // side operand (residual / dReLU aux) of the specialised epilogues: all column tiles issued
    // together here, one memory latency per tile instead of one per column tile
    constexpr bool kSideAll = (EMODE == SKC_EPI_RESID || EMODE == SKC_EPI_DRELU);
    float4 sdall[kSideAll ? NCT : 1][4];
    if constexpr (kSideAll) {
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
        const int64_t n = 32 * j + ec;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t mm = m0 + er + 8 * i;
          sdall[j][i] = ld4_or0(side, mm * p.sCm + n, mm < p.M && n + 3 < p.N);
        }
      }
    }
    bool rowok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t mm = m0 + er + 8 * i;
      rowok[i] = mm < p.M && epi_row_ok(p, mm < p.M ? mm : 0);
    }
    sk_wave_lds_sync();  // every slab read issued above has returned before Ep overwrites it
#pragma unroll
    for (int j = 0; j < NCT; ++j) {
      const int64_t n = 32 * j + ec;
      float4 sd4[4];  // side operand rows of this column tile (register budget: one tile at a time)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (kSideAll) {
          sd4[i] = sdall[j][i];
          continue;
        }
        const int64_t mm = m0 + er + 8 * i;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (side && n + 3 < p.N) {
          v = ld4_or0(side, mm * p.sCm + n, mm < p.M);
        } else if (side && mm < p.M && n < p.N) {
          v.x = side[mm * p.sCm + n];
          if (n + 1 < p.N) v.y = side[mm * p.sCm + n + 1];
          if (n + 2 < p.N) v.z = side[mm * p.sCm + n + 2];
        }
        sd4[i] = v;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) Ep[((i & 3) + 8 * (i >> 2) + 4 * h) * SK_EPS + r] = acc[j][i];
      sk_wave_lds_sync();
      const float bv[4] = {bn4[j].x, bn4[j].y, bn4[j].z, bn4[j].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = er + 8 * i;
        const int64_t mm = m0 + row;
        const float4 a = *reinterpret_cast<const float4*>(Ep + row * SK_EPS + ec);
        if (mm >= p.M || n >= p.N) continue;
        const float av4[4] = {a.x, a.y, a.z, a.w};
        const float s4[4] = {sd4[i].x, sd4[i].y, sd4[i].z, sd4[i].w};
        float o[4], pr[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = 0.f;
          pr[e] = 0.f;
          if (n + e < p.N)
            o[e] = skc_epi<EMODE>(p, mm, n + e, p.alpha * av4[e], bv[e], side ? s4[e] : 0.f, rowok[i], seed, keep_scale,
                             mse_part, pr[e]);
        }
        const int64_t off = mm * p.sCm + n;
        if (n + 3 < p.N) {
          *reinterpret_cast<float4*>(p.C + off) = make_float4(o[0], o[1], o[2], o[3]);
          if (epi & KDFM_EPI_STORE_PRE)
            *reinterpret_cast<float4*>(p.Cpre + off) = make_float4(pr[0], pr[1], pr[2], pr[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) {
              p.C[off + e] = o[e];
              if (epi & KDFM_EPI_STORE_PRE) p.Cpre[off + e] = pr[e];
            }
        }
      }
      sk_wave_lds_sync();  // Ep / the slab are rewritten next
    }
  }
  if (epi & KDFM_EPI_MSE) {
    mse_part = wave_sum(mse_part);
    if (lane == 0) atomicAdd(p.loss_acc, mse_part * p.loss_scale);
  }
}

template <int NCT, int EMODE = SKC_EPI_GENERIC>
int skc_launch(const GemmP& p, const SkGeo& g, int64_t gx, size_t lds, hipStream_t st) {
  static bool once = [] {
    hipFuncSetAttribute((const void*)skc_fwd_kernel<NCT, EMODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    return true;
  }();
  (void)once;
  set_route(ROUTE_SLAB_CONV);
  hipLaunchKernelGGL((skc_fwd_kernel<NCT, EMODE>), dim3((unsigned)gx), dim3(64 * SKC_WV), lds, st, p, g);
  return check_launch("kdfm_gemm(skinny conv slab)");
}

template <int NCT, int AMODE>
int skd_launch(const GemmP& p, const SkGeo& g, int G, int64_t gx, hipStream_t st) {
  hipLaunchKernelGGL((skd_fwd_kernel<NCT, AMODE>), dim3((unsigned)gx), dim3(256), 0, st, p, g, G);
  return check_launch("kdfm_gemm(skinny direct)");
}

template <int NCT, int AMODE, int WV, int EMODE = SKC_EPI_GENERIC>
int sk_launch(const GemmP& p, const SkGeo& g, int64_t gx, int64_t ncr, size_t lds, hipStream_t st) {
  if (lds > 64 * 1024) {
    static bool once = [] {
      hipFuncSetAttribute((const void*)sk_fwd_kernel<NCT, AMODE, WV, EMODE>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      return true;
    }();
    (void)once;
  }
  hipLaunchKernelGGL((sk_fwd_kernel<NCT, AMODE, WV, EMODE>), dim3((unsigned)gx, (unsigned)ncr), dim3(64 * WV), lds,
                     st, p, g);
  return check_launch("kdfm_gemm(skinny fwd)");
}

int env_int(const char* name, int dflt);

template <int AMODE, int WV>
int sk_dispatch_nct(int nct, const GemmP& p, const SkGeo& g, int64_t gx, int64_t ncr, size_t lds, hipStream_t st) {
  switch (nct) {
    case 1: return sk_launch<1, AMODE, WV>(p, g, gx, ncr, lds, st);
    case 2: return sk_launch<2, AMODE, WV>(p, g, gx, ncr, lds, st);
    default:
      if constexpr (AMODE == KDFM_LD_KC && WV == 4) {
        // the hot instantiation (stacked-head 1x1 convs / FM linears): compile-time epilogues
        static const int fast = env_int("KDFM_SKC_FAST_EPI", 1);
        switch ((fast && (p.N & 3) == 0 && (p.sCm & 3) == 0) ? skc_epi_mode(p.epi) : SKC_EPI_GENERIC) {
          case SKC_EPI_NONE: return sk_launch<3, AMODE, WV, SKC_EPI_NONE>(p, g, gx, ncr, lds, st);
          case SKC_EPI_RELU: return sk_launch<3, AMODE, WV, SKC_EPI_RELU>(p, g, gx, ncr, lds, st);
          case SKC_EPI_RESID: return sk_launch<3, AMODE, WV, SKC_EPI_RESID>(p, g, gx, ncr, lds, st);
          case SKC_EPI_DRELU: return sk_launch<3, AMODE, WV, SKC_EPI_DRELU>(p, g, gx, ncr, lds, st);
          case SKC_EPI_MSE: return sk_launch<3, AMODE, WV, SKC_EPI_MSE>(p, g, gx, ncr, lds, st);
          default: break;
        }
      }
      return sk_launch<3, AMODE, WV>(p, g, gx, ncr, lds, st);
  }
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

}  // namespace

int try_skinny_fwd(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st) {
  static const int enabled = env_int("KDFM_SKINNY", 1);
  static const int min_m = env_int("KDFM_SKINNY_MIN_M", 65536);
  static const int target_wgs = env_int("KDFM_SKINNY_WGS", 512);
  if (!enabled) return -1;
  if (batch != 1 || p.splitk != 1 || (p.epi & KDFM_EPI_ATOMIC) || p.ones_col >= 0) return -1;
  if (p.N <= 0 || p.K <= 0) return -1;
  if (bmode != KDFM_LD_KC && bmode != KDFM_LD_XC) return -1;
  if (p.sAk != 1 || (p.sAm & 3) || (((uintptr_t)p.A) & 15)) return -1;
  bool single;
  epi_side_src(p, single);
  if (!single) return -1;
  // row-major float4 epilogue: C (and R / aux / Cpre, laid out like C) 16-byte aligned rows
  if (p.sCn != 1 || (p.sCm & 3)) return -1;
  for (const void* q : {(const void*)p.C, (const void*)p.R, (const void*)p.aux, (const void*)p.Cpre})
    if (q && (((uintptr_t)q) & 15)) return -1;
  SkGeo g;
  if (amode == KDFM_LD_CONV) {
    if (p.conv_c % 16 != 0 || p.conv_c > SK_CHUNK || p.K != p.taps * p.conv_c || p.pad < 0 || p.pad >= p.taps)
      return -1;
    g.chunk = (int)p.conv_c;
    g.nchunks = p.taps;
  } else if (amode == KDFM_LD_KC) {
    if (p.K & 7) return -1;
    g.chunk = SK_CHUNK;
    g.nchunks = (int)ceil_div(p.K, SK_CHUNK);
  } else {
    return -1;
  }
  if (p.Bh && (p.K & 7) == 0 && (p.sBh & 7) == 0 && ((((uintptr_t)p.Bh) & 15) == 0)) {
    // measured slower than the generic 64x64 kernel on the 12,832-row encoder products
    // (fragment-shaped global loads, tools/shape_micro.py): opt-in only
    static const int direct_min_m = env_int("KDFM_SKINNY_DIRECT_MIN_M", 1 << 30);
    static const int direct_wgs = env_int("KDFM_SKINNY_DIRECT_WGS", 1024);
    if (p.M >= direct_min_m) {
      g.tiles = ceil_div(p.M, 32);
      const int64_t nt32 = ceil_div(p.N, 32);
      const int nct = nt32 <= 3 ? (int)nt32 : (nt32 % 3 == 0 || nt32 % 2 == 1) ? 3 : 2;
      const int G = (int)ceil_div(nt32, nct);
      int64_t gx = ceil_div(g.tiles * G, 4);
      if (gx > direct_wgs) gx = direct_wgs;
      if (amode == KDFM_LD_CONV) {
        switch (nct) {
          case 1: return skd_launch<1, KDFM_LD_CONV>(p, g, G, gx, st);
          case 2: return skd_launch<2, KDFM_LD_CONV>(p, g, G, gx, st);
          default: return skd_launch<3, KDFM_LD_CONV>(p, g, G, gx, st);
        }
      }
      switch (nct) {
        case 1: return skd_launch<1, KDFM_LD_KC>(p, g, G, gx, st);
        case 2: return skd_launch<2, KDFM_LD_KC>(p, g, G, gx, st);
        default: return skd_launch<3, KDFM_LD_KC>(p, g, G, gx, st);
      }
    }
  }
  if (p.M < min_m) return -1;
  g.Kp = (int)(ceil_div(p.K, 16) * 16);
  static const int slab = env_int("KDFM_SKINNY_CONV_SLAB", 1);
  static const int slab_wgs = env_int("KDFM_SKINNY_CONV_SLAB_WGS", 256);
  if (slab && amode == KDFM_LD_CONV && p.N <= 96 && p.conv_c <= SK_CHUNK && p.taps <= 3 && p.sAm >= p.conv_c) {
    // slab rows (32 + taps - 1) x conv_c must fit the SKC_SLAB_V registers / SKC_SLAB_BYTES of a wave
    g.ldb = g.Kp + 8;
    const int nct = (int)ceil_div(p.N, 32);
    g.gcols = 1;
    g.cw = 32 * nct;
    g.tiles = ceil_div(p.M, 32);
    const size_t lds = (size_t)g.cw * g.ldb * 2 + (size_t)SKC_WV * SKC_SLAB_BYTES;
    int64_t gx = ceil_div(g.tiles, SKC_WV);
    if (gx > slab_wgs) gx = slab_wgs;
    switch (nct) {
      case 1: return skc_launch<1>(p, g, gx, lds, st);
      case 2: return skc_launch<2>(p, g, gx, lds, st);
      default: {
        static const int fast = env_int("KDFM_SKC_FAST_EPI", 1);
        switch ((fast && (p.N & 3) == 0 && (p.sCm & 3) == 0) ? skc_epi_mode(p.epi) : SKC_EPI_GENERIC) {
          case SKC_EPI_RELU: return skc_launch<3, SKC_EPI_RELU>(p, g, gx, lds, st);
          case SKC_EPI_RESID: return skc_launch<3, SKC_EPI_RESID>(p, g, gx, lds, st);
          case SKC_EPI_DRELU: return skc_launch<3, SKC_EPI_DRELU>(p, g, gx, lds, st);
          default: return skc_launch<3>(p, g, gx, lds, st);
        }
      }
    }
  }
  if (amode == KDFM_LD_KC) {
    // the last chunk may read image columns up to nchunks*96 - 1: pad the image to that
    g.Kp = g.nchunks * SK_CHUNK;
  }
  g.ldb = g.Kp + 8;
  // column decomposition: NCT 32-col tiles per wave, gcols waves per row tile
  const int64_t nt32 = ceil_div(p.N, 32);
  int gcols, nct;
  if (nt32 <= 4) { gcols = 1; nct = (int)nt32; }
  else if (nt32 <= 8) { gcols = 2; nct = (int)ceil_div(nt32, 2); }
  else { gcols = 4; nct = (int)(nt32 <= 12 ? ceil_div(nt32, 4) : 3); }
  auto lds_of = [&](int gc, int nc) {
    return (size_t)32 * nc * gc * g.ldb * sizeof(uint16_t) + (size_t)4 * 32 * SK_EPS * sizeof(float);
  };
  const size_t lds_soft = 80 * 1024, lds_hard = 160 * 1024;
  while (lds_of(gcols, nct) > lds_soft && (nct > 1 || gcols > 1)) {
    if (nct > 1) --nct; else gcols >>= 1;
  }
  const size_t lds = lds_of(gcols, nct);
  if (lds > lds_hard) return -1;
  g.gcols = gcols;
  g.cw = 32 * nct * gcols;
  const int64_t ncr = ceil_div(p.N, g.cw);
  static const int max_ncr = env_int("KDFM_SKINNY_MAX_NCR", 2);
  if (ncr > max_ncr) return -1;  // A would be re-read more than max_ncr times: generic kernel
  g.tiles = ceil_div(p.M, 32);
  // waves per workgroup: enough workgroups to cover the CUs for small M, 4 waves otherwise
  int wv = 4;
  while (wv > gcols && (g.tiles * gcols) / wv * ncr < 256) wv >>= 1;
  if (wv < gcols) wv = gcols;
  const int rpi = wv / gcols;
  int64_t gx = ceil_div(g.tiles, rpi);
  const int64_t cap = ceil_div(target_wgs, ncr);
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  if (ncr > 65535) return -1;
  if (amode == KDFM_LD_CONV) {
    switch (wv) {
      case 1: return sk_dispatch_nct<KDFM_LD_CONV, 1>(nct, p, g, gx, ncr, lds, st);
      case 2: return sk_dispatch_nct<KDFM_LD_CONV, 2>(nct, p, g, gx, ncr, lds, st);
      default: return sk_dispatch_nct<KDFM_LD_CONV, 4>(nct, p, g, gx, ncr, lds, st);
    }
  }
  switch (wv) {
    case 1: return sk_dispatch_nct<KDFM_LD_KC, 1>(nct, p, g, gx, ncr, lds, st);
    case 2: return sk_dispatch_nct<KDFM_LD_KC, 2>(nct, p, g, gx, ncr, lds, st);
    default: return sk_dispatch_nct<KDFM_LD_KC, 4>(nct, p, g, gx, ncr, lds, st);
  }
}

}  // namespace kdfm
