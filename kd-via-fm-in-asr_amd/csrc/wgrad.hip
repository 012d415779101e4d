// Row-parallel weight gradients for the tall-skinny products of the ver5 step (bf16 MFMA, f32
// accumulate, deterministic ordered fold).
//
//   dW[m][n] (+)= alpha * sum_r dY[r][m] * X[r][n]      (+ the implicit ones column n = N-1 -> bias)
//
// Every Linear / 1x1 Conv1d weight gradient of the Conformer layers (12,832 rows at the bench
// shape, outputs up to 352 x 89) and of the layer-batched KD heads (205,312 rows, SimpleDenoiser's
// Conv1d(k=3) in CONV mode: X[r][n = tap*C + c] = x[r + tap - 1][c] inside each utterance;
// asr_train_diffm.py:400-460, 1295-1338) contracts over ALL rows into an output that fits one
// workgroup.  So each workgroup takes a contiguous run of rows and accumulates the WHOLE output (or a
// column slice of a very wide one) in MFMA accumulators: dY and X are each read from HBM exactly once,
// in 16-byte loads, and every workgroup writes one f32 partial; a fold kernel sums the partials in
// split order (one thread per output element: deterministic, no float atomics on the weight
// gradient).  The split-K generic kernel this replaces re-read the operands once per 64x64 output
// tile and added 25 partial sums per element with atomics.
//
// Pipeline: rows advance in 32-row steps (the MFMA K); step s+PD is loaded into registers while step
// s is multiplied out of LDS, so PD slabs of loads are in flight per workgroup.  Staging converts to
// bf16 and transposes into a [column][32 rows] LDS image (8-byte stores of 4 rows per column), from
// which A / B fragments are single 16-byte reads.
#include "gemm_common.h"

#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

// timing probe points (tools/wgrad_probe.hip defines KPROBE; empty in the library)
#ifndef KPROBE
#define KPROBE(i)
#endif

namespace kdfm {
namespace {

// explicit LDS (address space 3) views: generic pointers into the dynamic LDS array compiled to FLAT
// loads/stores, which also wait on the global-load counter and serialised the software pipeline
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T* lds_at(uint16_t* base, int off) {
  return reinterpret_cast<__attribute__((address_space(3))) T*>((lds_u16*)base + off);
}

constexpr int WR_NT = 512;      // threads: 8 waves, 2 per SIMD
constexpr int WR_LDK = 40;      // bf16 row stride of the [col][32 rows] image (80 B: conflict-light b128 reads)
constexpr int WR_MAXU = 2;      // staging units (4 rows x 4 cols) per thread per slab (template UPT <= this)

struct WrGeo {
  int wm, wn;        // wave grid over the block grid (wm * wn == 8)
  int Ma;            // A image columns: M padded to 16 * MBW * wm
  int Nb;            // B image columns of one slice (16 * NBW * wn)
  int64_t steps_per; // 32-row steps per split
  int64_t nmem;      // X columns in memory = ones_col if >= 0 else N
  int Msl;           // A columns (output rows) of one M slice (blockIdx.z), a multiple of 16
  int ascal;         // f32 A whose rows are not 16-byte aligned or M % 4 != 0 (the decoder's 129 classes):
                     // its staging units load 4 scalars each, columns past M masked to zero
  int xgrp;          // column slices of one split on one XCD (wr_block): they read the same rows
};

// (split, column slice) of this workgroup.  Workgroups go to the XCDs round-robin in dispatch order (x
// fastest), so with the plain grid the column slices of a split -- which read the same dY rows and (the
// strided conv gather) overlapping input rows -- land on different XCDs and fetch them through different
// L2s.  xgrp renumbers the grid in groups of 8 splits x all slices: dispatch slot L of a group goes to
// split 8 grp + (L % 8), slice L / 8, so a split's slices share the XCD L % 8 and run together; the
// splits past the last whole group keep the plain order.  A bijection of the grid (every partial is
// written by exactly one workgroup as before: results bitwise unchanged).
__device__ __forceinline__ void wr_block(const WrGeo& g, int& bx, int& by) {
  bx = (int)blockIdx.x;
  by = (int)blockIdx.y;
  if (!g.xgrp) return;
  const int S = (int)gridDim.x, nsl = (int)gridDim.y;
  const int L = bx + S * by, P = 8 * nsl, full = (S / 8) * P;
  if (L < full) {
    const int grp = L / P, r = L - grp * P;
    bx = grp * 8 + (r & 7);
    by = r >> 3;
  } else {
    const int t = L - full, rem = S - (S / 8) * 8;
    bx = (S / 8) * 8 + t % rem;
    by = t / rem;
  }
}

// BIN: dY and X are bf16 in memory (the fused KD-head chains store their saved operands as bf16,
// exactly the values the f32 path would round at staging), no conversion.  BIN = 1: staging units of
// 4 rows x 4 columns (8-byte loads); BIN = 2 (every column count a multiple of 8): 4 rows x 8 columns,
// 16-byte loads as in the f32 mode -- half the load instructions and half the units per slab, so
// the slab fits one unit per thread and two slabs stay in flight.
// C2D (BIN == 2 only): the B operand is gathered from a 3x3 stride-2 conv input (GemmP::c2_*) instead of a
// column matrix -- the striding subsampling's conv2 weight gradient without im2col
template <int MBW, int NBW, bool CONV, int PD, int UPT, int BIN = 0, bool C2D = false>
__global__ __launch_bounds__(WR_NT, 2) void wgr_kernel(GemmP p, WrGeo g) {
  static_assert(!C2D || (BIN == 2 && !CONV), "the conv gather stages 8-column bf16 units");
  constexpr int ES = BIN ? 2 : 4;   // element size in memory
  constexpr int CW = BIN == 2 ? 8 : 4;   // columns per staging unit
  constexpr int CWS = BIN == 2 ? 3 : 2;  // log2(CW)
  extern __shared__ __attribute__((aligned(16))) uint16_t wr_lds[];
  KPROBE(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // LDS images as element offsets into wr_lds (an array of pointers would decay to generic pointers
  // and turn every LDS access into a FLAT access that also waits on the global-load counter)
  const int ia = g.Ma * WR_LDK, ib = g.Nb * WR_LDK;   // image sizes (elements) of one buffer
  const int bufsz = ia + ib;                           // buffer b: A at b*bufsz, B at b*bufsz + ia
  // paired launch: blocks [S, 2S) compute the second product (same shape, its own operands / partials)
  int bx, by;
  wr_block(g, bx, by);
  const int64_t S_ = p.A2 ? (int64_t)gridDim.x / 2 : (int64_t)gridDim.x;
  const bool second = (int64_t)bx >= S_;
  const int64_t split = second ? (int64_t)bx - S_ : (int64_t)bx;
  const float* pA = second ? p.A2 : p.A;
  const float* pB = second ? p.B2 : p.B;
  float* pws = second ? p.ws2 : p.ws;
  const int64_t n0 = (int64_t)by * g.Nb;               // first output column of this slice
  // M slice: output rows m0 .. m0 + mcols - 1 (dY columns); more workgroups for short reductions
  // without growing any workgroup's partial
  const int m0 = (int)blockIdx.z * g.Msl;
  const int mcols = (p.M - m0 < g.Msl) ? (int)(p.M - m0) : g.Msl;
  const int64_t kb = split * g.steps_per * 32;
  int64_t ke = kb + g.steps_per * 32;
  if (ke > p.K) ke = p.K;
  if (p.k_dev) {   // rows decided on the device (compact step saves): the plan covers the capacity K
    const int64_t kd = *p.k_dev;
    if (ke > kd) ke = kd;
  }
  // B memory columns of this slice and the slab's staging units (4 rows x 4 columns each)
  const int ncols_mem = (int)((g.nmem - n0 < g.Nb) ? g.nmem - n0 : g.Nb);
  const int ma4 = (BIN == 0 && g.ascal) ? (mcols + CW - 1) >> CWS : mcols >> CWS;   // A column groups
  const int units = 8 * (ma4 + (ncols_mem >> CWS));

  // static image columns: A columns >= M and B columns beyond the memory columns are zero, the
  // ones column (bias gradient) is 1 in every row (rows past K contribute 0 through A)
  for (int e = threadIdx.x; e < 2 * (g.Ma + g.Nb) * 4; e += WR_NT) {
    const int buf = e / ((g.Ma + g.Nb) * 4);
    const int q = e - buf * (g.Ma + g.Nb) * 4;
    const int col = q >> 2, kq = (q & 3) * 8;
    int img;
    int c;
    bool zero = false, one = false;
    if (col < g.Ma) {
      img = buf * bufsz;
      c = col;
      zero = c >= mcols;
    } else {
      img = buf * bufsz + ia;
      c = col - g.Ma;
      const int64_t n = n0 + c;
      one = p.nseg <= 1 && p.ones_col >= 0 && n == p.ones_col;   // segment columns: per slab (stage)
      const bool segc = p.nseg > 1 && n >= p.ones_col && n < p.ones_col + p.nseg;   // written by stage()
      zero = !one && !segc && (c >= ncols_mem);
    }
    if (zero || one) {
      const uint16_t v = one ? (uint16_t)0x3F80 : (uint16_t)0;  // bf16(1.0) = 0x3F80
      bf16x8 pk;
#pragma unroll
      for (int i = 0; i < 8; ++i) pk[i] = (short)v;
      *lds_at<bf16x8>(wr_lds, img + c * WR_LDK + kq) = pk;
    }
  }

  // staging unit u: row group rg = u % 8 (rows 4rg..4rg+3 of a slab), column group cg = u / 8 (4
  // consecutive columns of A (cg < ma4) or of B).  Per-unit source pointers and (CONV) frame
  // counters are set up once and advanced by one slab per step: no 64-bit multiplies in the loop.
  // Rows past the split's end or outside the utterance (CONV taps) load from a clamped valid address
  // and are zeroed by a select (branch-free).
  const char* src[UPT];   // byte pointers (ES-byte elements)
  int acol[UPT];          // ascal: the unit's first A column (>= mcols: not an A unit)
  int64_t ld[UPT];        // row stride in bytes
  int tfr[UPT], toff[UPT];   // CONV: frame of the unit's first row in its utterance; tap - pad
  bool act[UPT];
  // C2D B units: tap offsets, channel and the (utterance, t2, f2) position of the unit's first row
  int c2ky[UPT], c2kx[UPT], c2c[UPT], c2f[UPT], c2t[UPT], c2b[UPT];
  int c2l0[UPT], c2l1[UPT];   // frame limits of utterances c2b and c2b + 1 (a slab's rows span at most two)
  bool c2u[UPT];
  auto c2lim = [&](int bb) -> int {
    const int64_t nb = p.K / (p.c2_T2 * p.c2_F2);
    if (bb >= nb) return 0;
    return (int)(p.c2_len ? min(p.c2_len[bb], p.c2_T1) : p.c2_T1);
  };
#pragma unroll
  for (int i = 0; i < UPT; ++i) {
    const int u = threadIdx.x + i * WR_NT;
    act[i] = u < units;
    const int rg = u & 7, cg = act[i] ? (u >> 3) : 0;
    const int64_t r0 = kb + rg * 4;
    tfr[i] = 0;
    toff[i] = 0;
    acol[i] = 1 << 30;
    c2u[i] = false;
    c2ky[i] = c2kx[i] = c2c[i] = c2f[i] = c2t[i] = c2b[i] = c2l0[i] = c2l1[i] = 0;
    if (cg < ma4) {
      src[i] = reinterpret_cast<const char*>(pA) + ES * (r0 * p.sAk + m0 + cg * CW);
      ld[i] = ES * p.sAk;
      acol[i] = cg * CW;
    } else {
      const int64_t n = n0 + (int64_t)(cg - ma4) * CW;
      ld[i] = ES * p.sBk;
      if constexpr (CONV) {
        const int64_t tap = n / p.conv_c, c = n - tap * p.conv_c;
        toff[i] = (int)(tap - p.pad);
        tfr[i] = (int)(r0 % p.conv_t);
        src[i] = reinterpret_cast<const char*>(pB) + ES * ((r0 + toff[i]) * p.sBk + c);
      } else if constexpr (C2D) {
        const int64_t tap = n / p.conv_c;
        ld[i] = 0;
        c2u[i] = true;
        c2ky[i] = (int)(tap / 3);
        c2kx[i] = (int)(tap - 3 * (tap / 3));
        c2c[i] = (int)(n - tap * p.conv_c);
        c2f[i] = (int)(r0 % p.c2_F2);
        c2t[i] = (int)((r0 / p.c2_F2) % p.c2_T2);
        c2b[i] = (int)(r0 / (p.c2_F2 * p.c2_T2));
        c2l0[i] = c2lim(c2b[i]);
        c2l1[i] = c2lim(c2b[i] + 1);
        src[i] = reinterpret_cast<const char*>(pB);
      } else {
        src[i] = reinterpret_cast<const char*>(pB) + ES * (r0 * p.sBk + n);
      }
    }
  }
  const int T = CONV ? (int)p.conv_t : 0;
  float4 reg[PD][UPT][4];
  uint32_t msk[PD];   // bit i*4+j: row j of unit i is real data (else staged as 0)
  // k0: first row of the slab (uniform); the unit pointers already point at it.  The loads go
  // straight into the slab registers and the validity select is applied at staging time: a select
  // right after a load would make every load wait for its own data (no loads in flight across steps).
  auto load = [&](float4 (&r)[UPT][4], uint32_t& m, int64_t k0) {
    const bool full = k0 + 32 <= ke;
    m = 0u;
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bool ok = act[i];
        if (!full) ok = ok && (k0 + (threadIdx.x & 7) * 4 + j < ke);
        if constexpr (CONV) {
          if (ok) {   // frame of row j within the utterance, shifted by the tap
            int t = tfr[i] + j;
            t = (t >= T) ? t - T : t;
            const int tt = t + toff[i];
            ok = tt >= 0 && tt < T;
          }
        }
        const char* q = ok ? src[i] + j * ld[i] : reinterpret_cast<const char*>(pB);   // any valid, aligned address
        if constexpr (C2D) {
          if (c2u[i]) {   // output position of row j -> the tap's input position (zero outside / past len)
            int f2 = c2f[i] + j, t2 = c2t[i], bb = c2b[i];
            if (f2 >= (int)p.c2_F2) {
              f2 -= (int)p.c2_F2;
              if (++t2 >= (int)p.c2_T2) {
                t2 = 0;
                ++bb;
              }
            }
            const int t1 = 2 * t2 - 1 + c2ky[i], f1 = 2 * f2 - 1 + c2kx[i];
            const int lim = bb == c2b[i] ? c2l0[i] : c2l1[i];
            ok = ok && t1 >= 0 && t1 < lim && f1 >= 0 && f1 < p.c2_F1;
            q = ok ? reinterpret_cast<const char*>(pB) +
                         ES * ((((int64_t)bb * p.c2_T1 + t1) * p.c2_F1 + f1) * p.c2_ld + c2c[i])
                   : reinterpret_cast<const char*>(pB);
          }
        }
        if constexpr (BIN == 1) {
          const uint2 t = *reinterpret_cast<const uint2*>(q);
          r[i][j] = make_float4(__builtin_bit_cast(float, t.x), __builtin_bit_cast(float, t.y), 0.f, 0.f);
        } else if constexpr (BIN == 0) {
          if (g.ascal && acol[i] < mcols) {   // unaligned A row: 4 scalar loads, columns past M clamped + zeroed
            const float* qa = reinterpret_cast<const float*>(q);
            const int cb = acol[i];
            float e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) e[k] = qa[cb + k < mcols ? k : 0] * (cb + k < mcols ? 1.f : 0.f);
            r[i][j] = make_float4(e[0], e[1], e[2], e[3]);
          } else {
            r[i][j] = *reinterpret_cast<const float4*>(q);
          }
        } else {
          r[i][j] = *reinterpret_cast<const float4*>(q);
        }
        m |= (ok ? 1u : 0u) << (i * 4 + j);
      }
      src[i] += 32 * ld[i];
      if constexpr (CONV) {
        tfr[i] += 32;
        while (tfr[i] >= T) tfr[i] -= T;
      }
      if constexpr (C2D) {   // the next slab's first row
        c2f[i] += 32;
        while (c2f[i] >= (int)p.c2_F2) {
          c2f[i] -= (int)p.c2_F2;
          if (++c2t[i] >= (int)p.c2_T2) {
            c2t[i] = 0;
            ++c2b[i];
            c2l0[i] = c2l1[i];
            c2l1[i] = c2lim(c2b[i] + 1);   // needed from the next slab on: the wait lands there
          }
        }
      }
    }
  };
  auto stage = [&](const float4 (&r)[UPT][4], uint32_t m, int buf, int64_t k0) {
    if (p.nseg > 1) {
      // per-segment ones columns (a slab never straddles segments: seg_rows % 32 == 0): column
      // ones_col + j is 1 in the slab's rows iff the slab lies in segment j
      const int t = threadIdx.x;
      if (t < 4 * p.nseg) {
        const int sc = t >> 2;
        const uint16_t v = (sc == (int)(k0 / p.seg_rows)) ? (uint16_t)0x3F80 : (uint16_t)0;
        bf16x8 pk;
#pragma unroll
        for (int i = 0; i < 8; ++i) pk[i] = (short)v;
        *lds_at<bf16x8>(wr_lds, buf * bufsz + ia + (int)(p.ones_col - n0 + sc) * WR_LDK + (t & 3) * 8) = pk;
      }
    }
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int u = threadIdx.x + i * WR_NT;
      if (u >= units) continue;
      const int rg = u & 7, cg = u >> 3;
      int img, c0;
      if (cg < ma4) {
        img = buf * bufsz;
        c0 = cg * CW;
      } else {
        img = buf * bufsz + ia;
        c0 = (cg - ma4) * CW;
      }
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 v0 = ((m >> (i * 4 + 0)) & 1u) ? r[i][0] : z;
      const float4 v1 = ((m >> (i * 4 + 1)) & 1u) ? r[i][1] : z;
      const float4 v2 = ((m >> (i * 4 + 2)) & 1u) ? r[i][2] : z;
      const float4 v3 = ((m >> (i * 4 + 3)) & 1u) ? r[i][3] : z;
      if constexpr (BIN == 2) {
        // row j's 8 bf16 columns: column q is half (q & 1) of dword q >> 1; the 4 rows of a column
        // pair up by byte permutes (low halves: selector 0x05040100, high halves: 0x07060302)
        const uint32_t w[4][4] = {{__builtin_bit_cast(uint32_t, v0.x), __builtin_bit_cast(uint32_t, v0.y),
                                   __builtin_bit_cast(uint32_t, v0.z), __builtin_bit_cast(uint32_t, v0.w)},
                                  {__builtin_bit_cast(uint32_t, v1.x), __builtin_bit_cast(uint32_t, v1.y),
                                   __builtin_bit_cast(uint32_t, v1.z), __builtin_bit_cast(uint32_t, v1.w)},
                                  {__builtin_bit_cast(uint32_t, v2.x), __builtin_bit_cast(uint32_t, v2.y),
                                   __builtin_bit_cast(uint32_t, v2.z), __builtin_bit_cast(uint32_t, v2.w)},
                                  {__builtin_bit_cast(uint32_t, v3.x), __builtin_bit_cast(uint32_t, v3.y),
                                   __builtin_bit_cast(uint32_t, v3.z), __builtin_bit_cast(uint32_t, v3.w)}};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t sel = (q & 1) ? 0x07060302u : 0x05040100u;
          const uint32_t lo = __builtin_amdgcn_perm(w[1][q >> 1], w[0][q >> 1], sel);
          const uint32_t hi = __builtin_amdgcn_perm(w[3][q >> 1], w[2][q >> 1], sel);
          *lds_at<u32x2>(wr_lds, img + (c0 + q) * WR_LDK + rg * 4) = u32x2{lo, hi};
        }
      } else if constexpr (BIN == 1) {
        // row j's 4 bf16 columns: (q0 | q1 << 16) in .x, (q2 | q3 << 16) in .y
        const uint32_t w[4][2] = {{__builtin_bit_cast(uint32_t, v0.x), __builtin_bit_cast(uint32_t, v0.y)},
                                  {__builtin_bit_cast(uint32_t, v1.x), __builtin_bit_cast(uint32_t, v1.y)},
                                  {__builtin_bit_cast(uint32_t, v2.x), __builtin_bit_cast(uint32_t, v2.y)},
                                  {__builtin_bit_cast(uint32_t, v3.x), __builtin_bit_cast(uint32_t, v3.y)}};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int sh = 16 * (q & 1);
          const uint32_t b0 = (w[0][q >> 1] >> sh) & 0xFFFFu, b1 = (w[1][q >> 1] >> sh) & 0xFFFFu;
          const uint32_t b2 = (w[2][q >> 1] >> sh) & 0xFFFFu, b3 = (w[3][q >> 1] >> sh) & 0xFFFFu;
          *lds_at<u32x2>(wr_lds, img + (c0 + q) * WR_LDK + rg * 4) = u32x2{b0 | (b1 << 16), b2 | (b3 << 16)};
        }
      } else {
        const float* f0 = reinterpret_cast<const float*>(&v0);
        const float* f1 = reinterpret_cast<const float*>(&v1);
        const float* f2 = reinterpret_cast<const float*>(&v2);
        const float* f3 = reinterpret_cast<const float*>(&v3);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t lo = pack_bf16x2(f0[q], f1[q]);
          const uint32_t hi = pack_bf16x2(f2[q], f3[q]);
          *lds_at<u32x2>(wr_lds, img + (c0 + q) * WR_LDK + rg * 4) = u32x2{lo, hi};
        }
      }
    }
  };

  const int wr_ = wave / g.wn, wc_ = wave - (wave / g.wn) * g.wn;
  const int mb0 = wr_ * MBW, nb0 = wc_ * NBW;
  f32x4 acc[MBW][NBW];
#pragma unroll
  for (int i = 0; i < MBW; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t nsteps = (ke > kb) ? (ke - kb + 31) / 32 : 0;
  auto mfma_step = [&](int buf) {
    const int oA = buf * bufsz, oB = buf * bufsz + ia;
    bf16x8 af[MBW];
#pragma unroll
    for (int i = 0; i < MBW; ++i)
      af[i] = *lds_at<bf16x8>(wr_lds, oA + ((mb0 + i) * 16 + (lane & 15)) * WR_LDK + 8 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const bf16x8 bfr = *lds_at<bf16x8>(wr_lds, oB + ((nb0 + j) * 16 + (lane & 15)) * WR_LDK + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < MBW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (PD == 1) {
    if (nsteps > 0) {
      load(reg[0], msk[0], kb);
      stage(reg[0], msk[0], 0, kb);
    }
    __syncthreads();
    int buf = 0;
    for (int64_t s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) load(reg[0], msk[0], kb + 32 * (s + 1));
      mfma_step(buf);
      if (s + 1 < nsteps) stage(reg[0], msk[0], buf ^ 1, kb + 32 * (s + 1));
      __syncthreads();
      buf ^= 1;
    }
  } else {
    // two slabs in flight: slot 0 carries even steps, slot 1 odd steps (compile-time slots, so the
    // compiler waits only for the older slot's loads before staging it)
    KPROBE(1);
    if (nsteps > 0) load(reg[0], msk[0], kb);
    if (nsteps > 1) load(reg[1], msk[1], kb + 32);
    if (nsteps > 0) stage(reg[0], msk[0], 0, kb);
    __syncthreads();
    KPROBE(2);
    for (int64_t s = 0; s < nsteps; s += 2) {
      // even step s in buffer 0
      if (s + 2 < nsteps) load(reg[0], msk[0], kb + 32 * (s + 2));
      mfma_step(0);
      if (s + 1 < nsteps) stage(reg[1], msk[1], 1, kb + 32 * (s + 1));
      __syncthreads();
      if (s + 1 >= nsteps) break;
      // odd step s+1 in buffer 1
      if (s + 3 < nsteps) load(reg[1], msk[1], kb + 32 * (s + 3));
      mfma_step(1);
      if (s + 2 < nsteps) stage(reg[0], msk[0], 0, kb + 32 * (s + 2));
      __syncthreads();
      if (s < 40) KPROBE(3 + (int)(s >> 1));
    }
  }
  KPROBE(29);

  if (p.xslots) {
    // non-deterministic mode: add into the slot of the XCD this workgroup runs on (HW_REG_XCC_ID; the
    // slot choice is locality only -- the adds are device-coherent atomics wherever they land), so the
    // partial traffic is 8 slots in L2 instead of one f32 tile per split through HBM
    const int xcd = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;
    float* wsx = pws + (int64_t)xcd * p.M * p.N;
#pragma unroll
    for (int i = 0; i < MBW; ++i)
#pragma unroll
      for (int j = 0; j < NBW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = (mb0 + i) * 16 + (lane >> 4) * 4 + r;
          const int64_t n = n0 + (nb0 + j) * 16 + (lane & 15);
          if (ml < mcols && n < p.N && n < n0 + g.Nb)
            __hip_atomic_fetch_add(wsx + (m0 + ml) * p.N + n, acc[i][j][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    return;
  }
  // raw partial of this (split, slice) -> ws[split][m][n]
  float* wsp = pws + split * p.M * p.N;
#pragma unroll
  for (int i = 0; i < MBW; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ml = (mb0 + i) * 16 + (lane >> 4) * 4 + r;
        const int64_t n = n0 + (nb0 + j) * 16 + (lane & 15);
        if (ml < mcols && n < p.N && n < n0 + g.Nb) wsp[(m0 + ml) * p.N + n] = acc[i][j][r];
      }
  KPROBE(31);
}

// C(m, n) += alpha * sum_{s<S} ws[s][m][n]   (n == ones_col -> ones_out[m]), deterministic: the block
// owns 64 consecutive output elements (lane = element: coalesced partial rows), its 8 waves take the
// splits s = w, w+8, ... with 4 independent accumulators each (many loads in flight: the fold is
// latency-bound otherwise), then a fixed-order combine in LDS and one plain add per element.
constexpr int WF_WAVES = 8;

template <bool TRANS = false>   // TRANS: partials stored ws[s][n][m] (wgd_kernel)
__global__ __launch_bounds__(64 * WF_WAVES) void wgr_fold_kernel(GemmP p, int64_t S) {
  __shared__ float red[WF_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t MN = p.M * p.N;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const bool second = blockIdx.y == 1;   // paired launch: the second product
  const float* ws = second ? p.ws2 : p.ws;
  float* Cout = second ? p.C2 : p.C;
  float* ones = second ? p.ones_out2 : p.ones_out;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (e < MN) {
    int64_t s = w;
    for (; s + 3 * WF_WAVES < S; s += 4 * WF_WAVES) {
      a0 += ws[s * MN + e];
      a1 += ws[(s + WF_WAVES) * MN + e];
      a2 += ws[(s + 2 * WF_WAVES) * MN + e];
      a3 += ws[(s + 3 * WF_WAVES) * MN + e];
    }
    for (; s < S; s += WF_WAVES) a0 += ws[s * MN + e];
  }
  red[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && e < MN) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < WF_WAVES; ++i) v += red[i][lane];
    v *= p.alpha;
    int64_t m, n;
    if (TRANS) {
      n = e / p.M;
      m = e - n * p.M;
    } else {
      m = e / p.N;
      n = e - m * p.N;
    }
    if (p.ones_col >= 0 && n >= p.ones_col)   // bias column(s): segment j -> ones_out[j][m]
      ones[(n - p.ones_col) * p.M + m] += v;
    else
      Cout[m * p.sCm + n * p.sCn] += v;
  }
}

// The same fold with 4 consecutive output elements per lane (16-byte partial loads; M*N % 4 == 0): a block
// owns 256 elements, so the launch has a quarter of the blocks and every load instruction moves 4x the
// bytes -- the fold is load-issue bound (r4k: 162 launches per step at 7.3 us each).  One block's work as a
// device function: the per-product kernel below and the batched fold (wgr_fold_batch_kernel) both run it.
__device__ __forceinline__ void fold4_block(const float* __restrict__ ws_base, float* Cout, float* ones, int64_t M,
                                            int64_t N, int64_t sCm, int64_t sCn, int64_t ones_col, float alpha,
                                            int64_t S, bool trans, int64_t blk, float4 (*red4)[64]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t MN = M * N;
  const int64_t e0 = (blk * 64 + lane) * 4;
  // wave 0 fetches the 4 destination values before the partials, so their round trip overlaps the
  // partials' (the destination is read and written by this block only)
  float* dst[4] = {nullptr, nullptr, nullptr, nullptr};
  float cur[4] = {0.f, 0.f, 0.f, 0.f};
  if (w == 0 && e0 < MN) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = e0 + q;
      int64_t m, n;
      if (trans) {
        n = e / M;
        m = e - n * M;
      } else {
        m = e / N;
        n = e - m * N;
      }
      dst[q] = (ones_col >= 0 && n >= ones_col) ? ones + (n - ones_col) * M + m : Cout + m * sCm + n * sCn;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = *dst[q];
  }
  float4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [](float4& a, const float4 b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; };
  // this wave's splits w, w + WF, ... (nw of them): split i of the wave goes to accumulator i % 4 while it is
  // in a complete group of 4 (i < g4), the rest to accumulator 0 -- a fixed order.  Up to 16 partial loads
  // are in flight per lane before the first add (one memory round trip per 16 splits, not per 4).
  const int64_t nw = (e0 < MN && S > w) ? (S - w + WF_WAVES - 1) / WF_WAVES : 0;
  const int64_t g4 = nw / 4 * 4;
  const float4* base = reinterpret_cast<const float4*>(ws_base + e0);
  const int64_t st = MN / 4;   // float4 stride between splits
  for (int64_t i0 = 0; i0 < nw; i0 += 16) {
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      v[i] = i0 + i < nw ? base[(w + (i0 + i) * WF_WAVES) * st] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i0 + i < nw) add(i0 + i < g4 ? acc[i & 3] : acc[0], v[i]);
    }
  }
  add(acc[0], acc[1]);
  add(acc[2], acc[3]);
  add(acc[0], acc[2]);
  red4[w][lane] = acc[0];
  __syncthreads();
  if (w == 0 && e0 < MN) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < WF_WAVES; ++i) add(v, red4[i][lane]);
    const float vv[4] = {v.x * alpha, v.y * alpha, v.z * alpha, v.w * alpha};
#pragma unroll
    for (int q = 0; q < 4; ++q) *dst[q] = cur[q] + vv[q];
  }
}

template <bool TRANS = false>
__global__ __launch_bounds__(64 * WF_WAVES) void wgr_fold4_kernel(GemmP p, int64_t S) {
  __shared__ float4 red4[WF_WAVES][64];
  const bool second = blockIdx.y == 1;   // paired launch: the second product
  fold4_block(second ? p.ws2 : p.ws, second ? p.C2 : p.C, second ? p.ones_out2 : p.ones_out, p.M, p.N, p.sCm, p.sCn,
              p.ones_col, p.alpha, S, TRANS, blockIdx.x, red4);
}

// Deferred folds (kdfm_wgrad_set_fold_arena / kdfm_wgrad_fold_flush): the row-parallel products of a stream
// write their partials into a caller-owned arena and queue a fold job each; one launch then folds every
// queued product (block ranges per job), each job exactly as its own wgr_fold4_kernel launch would (the
// same fold4_block: bitwise equal results).  A Conformer layer's 8 weight gradients fold in one launch
// instead of 6 (114 fold launches per step, 8-11 us each, mostly ramp and tail).
constexpr int FB_MAXJ = 24;
struct FoldJob {
  const float* ws; float* C; float* ones;
  int64_t M, N, sCm, sCn, ones_col, S;
  float alpha; int trans;
};
struct FoldBatch {
  FoldJob j[FB_MAXJ];
  int64_t blk0[FB_MAXJ + 1];   // first block of each job; blk0[n] = grid
  int n;
};

__global__ __launch_bounds__(64 * WF_WAVES) void wgr_fold_batch_kernel(FoldBatch fb) {
  __shared__ float4 red4[WF_WAVES][64];
  const int64_t b = blockIdx.x;
  int j = 0;
  while (j + 1 < fb.n && b >= fb.blk0[j + 1]) ++j;   // block-uniform
  const FoldJob& J = fb.j[j];
  fold4_block(J.ws, J.C, J.ones, J.M, J.N, J.sCm, J.sCn, J.ones_col, J.alpha, J.S, J.trans != 0, b - fb.blk0[j], red4);
}

// fold launch: the 4-wide kernel when the partial layout allows it (KDFM_WGR_FOLD4=0: the scalar one)
template <bool TRANS>
void fold_launch(const GemmP& p, int64_t S, hipStream_t st) {
  static const int f4 = [] { const char* e = getenv("KDFM_WGR_FOLD4"); return e ? atoi(e) : 1; }();
  const int64_t MN = p.M * p.N;
  const unsigned np = p.A2 ? 2u : 1u;
  if (f4 && MN % 4 == 0 && (((uintptr_t)p.ws | (uintptr_t)p.ws2) & 15) == 0)
    hipLaunchKernelGGL(wgr_fold4_kernel<TRANS>, dim3((unsigned)ceil_div(MN, 256), np), dim3(64 * WF_WAVES), 0, st, p, S);
  else
    hipLaunchKernelGGL(wgr_fold_kernel<TRANS>, dim3((unsigned)ceil_div(MN, 64), np), dim3(64 * WF_WAVES), 0, st, p, S);
}

struct WrPick { int mbw, nbw, wm, wn; };

// per-wave block counts among the compiled instances (3,2) (3,3) (3,4) (3,6) (6,3), 8 waves
bool wr_pick(int64_t M, int64_t Ncols, WrPick& w) {
  const int64_t Mb = ceil_div(M, 16), Nb = ceil_div(Ncols, 16);
  static const int shapes[5][2] = {{3, 2}, {3, 3}, {3, 4}, {3, 6}, {6, 3}};
  static const int grids[4][2] = {{1, 8}, {2, 4}, {4, 2}, {8, 1}};
  int best = 1 << 30;
  for (auto& gr : grids)
    for (auto& sh : shapes) {
      if ((int64_t)sh[0] * gr[0] < Mb || (int64_t)sh[1] * gr[1] < Nb) continue;
      const int cost = sh[0] * sh[1] * 4 + (sh[0] + sh[1]);   // MFMA slots (incl. padding) + fragment reads
      if (cost < best) {
        best = cost;
        w = {sh[0], sh[1], gr[0], gr[1]};
      }
    }
  return best < (1 << 30);
}

int env_i(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// geometry of wgd_kernel (bf16 operands streamed by LDS-DMA, below)
struct WdGeo {
  int wm, wn;            // wave grid
  int Mt, Nt;            // 16-wide tiles of M and of X's memory columns
  int64_t steps_per;     // 32-row slabs per split
  int pa, pb, pw;        // 1 KB DMA pieces of a slab's dY / X image, DMA instructions per wave per slab
  int aimg, slab;        // bf16 elements of the (1 KB padded) dY image and of one slab buffer
};

// private B-operand mode of the row-parallel kernel: the 3x3 stride-2 conv gather (GemmP::c2_*)
constexpr int WR_LD_C2D = 16;
inline int64_t nmem_c2d(const GemmP& p) { return p.ones_col >= 0 ? p.ones_col : p.N; }

struct WrPlan {
  WrPick w;
  WrGeo g;
  int64_t S, slices, mslices;
  size_t lds;
  int upt;
  int bin;   // wgr_kernel BIN: 0 f32 operands, 1 / 2 bf16 operands in 4- / 8-column staging units
  bool dma = false;   // wgd_kernel route
  int ns = 0;         // wgd_kernel slab buffers
  WdGeo wd{};
};

bool wd_plan(const GemmP& p, int bmode, WrPlan& pl);

bool wr_plan(const GemmP& p, int amode, int bmode, int64_t batch, WrPlan& pl, bool force = false,
             bool bf16in = false) {
  if (bf16in && force && batch == 1 && amode == KDFM_LD_XC && wd_plan(p, bmode, pl)) return true;
  static const int enabled = env_i("KDFM_WGR", 1);
  if (!enabled && !force) return false;
  if (batch != 1 || p.epi != KDFM_EPI_ATOMIC || amode != KDFM_LD_XC) return false;
  if (bmode != KDFM_LD_XC && bmode != KDFM_LD_CONV && bmode != WR_LD_C2D) return false;
  if (bmode == WR_LD_C2D && (!bf16in || (p.conv_c & 7) || p.M % 8 || p.sAk % 8 || nmem_c2d(p) != 9 * p.conv_c ||
                             p.c2_T2 != (p.c2_T1 - 1) / 2 + 1 || p.c2_F2 != (p.c2_F1 - 1) / 2 + 1 || p.c2_F2 < 4))
    return false;
  // f32 A rows that are not 16-byte aligned (or M % 4 != 0): scalar A staging (WrGeo::ascal)
  const bool ascal = !bf16in && ((p.sAk & 3) || (p.M & 3) || (((uintptr_t)p.A) & 15));
  if (p.sAm != 1 || (bf16in && ((p.sAk & 3) || (p.M & 3) || (((uintptr_t)p.A) & 15)))) return false;
  if (ascal && (((uintptr_t)p.A) & 3)) return false;
  if (p.sBn != 1 || (p.sBk & 3) || (((uintptr_t)p.B) & 15)) return false;
  const int nseg = p.nseg > 1 ? p.nseg : 1;
  if (p.ones_col >= 0 && p.ones_col != p.N - nseg) return false;
  if (nseg > 1 && (p.ones_col < 0 || nseg > 16 || p.seg_rows <= 0 || p.seg_rows % 32 || p.K != nseg * p.seg_rows))
    return false;
  const int64_t nmem = p.ones_col >= 0 ? p.ones_col : p.N;
  if (nmem & 3) return false;
  if (bmode == KDFM_LD_CONV && ((p.conv_c & 3) || p.taps < 1 || p.pad < 0 || nmem != p.taps * p.conv_c)) return false;
  static const int min_k = env_i("KDFM_WGR_MINK", 512);
  if (p.K < min_k && !force) return false;
  // column slices of at most 24 16-wide blocks (a (6,3) wave tile on a 1x8 wave grid)
  const int64_t Nb_all = ceil_div(p.N, 16);
  pl.slices = ceil_div(Nb_all, 24);
  if (nseg > 1 && pl.slices != 1) return false;   // the segment columns live in the one slice
  const int64_t ncols_slice = ceil_div(Nb_all, pl.slices) * 16;
  // short reductions (the 12,832-row Conformer products: S is capped by min_steps, 66 splits)
  // leave most of the 256 CUs idle; slice the output rows too, so every CU gets a workgroup while
  // each workgroup's partial (and the fold's input) shrinks with its slice
  const int64_t steps = ceil_div(p.K, 32);
  // workgroup target.  Isolated, two per CU is faster for the non-CONV products (FM dW2 at 1.64M
  // rows 247 -> 164 us, tools/gpu_wgr_wgs.sh, profiles/r02/wgs_*.log); inside the step, where these
  // run on the weight-gradient stream beside the critical-path kernels, one per CU wins (bench
  // 1655 -> 1686 utt/s, tools/gpu_wgr_env_ab.sh, profiles/r02/envab_*.log)
  static const int target_all = env_i("KDFM_WGR_WGS", 256);
  // conv-mode products (the denoiser's k=3 convs over the stacked head rows, 4 per step) may take fewer
  // workgroups so the compute stream's heads kernels keep CUs beside them (KDFM_WGR_CONV_WGS)
  static const int target_conv = env_i("KDFM_WGR_CONV_WGS", target_all);
  // the striding subsampling's conv2 weight gradient (WR_LD_C2D) runs at the step's tail beside the conv2 data
  // gradient, where nothing else waits for CUs: its 256 640 rows over 3 column slices get more, shorter splits
  static const int target_c2d = env_i("KDFM_WGR_C2D_WGS", target_all);
  const int target = bmode == KDFM_LD_CONV ? target_conv : bmode == WR_LD_C2D ? target_c2d : target_all;
  // at least 6 32-row steps per split: the 12 832-row products take 66 splits (4 -> 100 splits: 2303-2309 utt/s,
  // 6: 2318-2325, 8: 2316-2318, 12: 2255, 16: 2150 -- profiles/r05/r5zh, r5zi; fewer partial bytes until the
  // longer per-workgroup chains delay the weight-gradient stream's tail)
  static const int min_steps = env_i("KDFM_WGR_STEPS", 6);
  // off by default: isolated the slices help (FFN W1 25 -> 19 us) but in the step the extra
  // workgroups queue behind the critical-path kernels (bench 1687 unsliced vs 1635 sliced at
  // target 256, profiles/r02/envab_*.log).  Read per call: tests compare sliced / unsliced.
  const int msl_on = env_i("KDFM_WGR_MSL", 0);
  const int64_t smax = steps / min_steps > 0 ? steps / min_steps : 1;
  {
    const int64_t s0 = target / pl.slices < 1 ? 1 : target / pl.slices;
    const int64_t s_est = s0 < smax ? s0 : smax;
    int64_t ms = msl_on ? target / (s_est * pl.slices) : 1;
    const int64_t ms_cap = p.M / 32;   // slices of at least 32 output rows
    if (ms > ms_cap) ms = ms_cap;
    if (ms < 1) ms = 1;
    pl.g.Msl = (int)(ceil_div(ceil_div(p.M, ms), 16) * 16);
    pl.mslices = ceil_div(p.M, pl.g.Msl);
  }
  if (!wr_pick(pl.g.Msl, ncols_slice, pl.w)) return false;
  const int bin8 = env_i("KDFM_WGR_BIN8", 1);   // per call, like KDFM_WGR_MSL
  pl.bin = !bf16in ? 0
           : (bin8 && p.M % 8 == 0 && nmem % 8 == 0 && p.sAk % 8 == 0 && p.sBk % 8 == 0 &&
              (bmode != KDFM_LD_CONV || p.conv_c % 8 == 0)) ? 2 : 1;
  if (bmode == WR_LD_C2D && pl.bin != 2) return false;
  const int cw = pl.bin == 2 ? 8 : 4;
  pl.g.wm = pl.w.wm;
  pl.g.wn = pl.w.wn;
  pl.g.Ma = 16 * pl.w.mbw * pl.w.wm;
  pl.g.Nb = 16 * pl.w.nbw * pl.w.wn;
  pl.slices = ceil_div(p.N, pl.g.Nb);
  pl.g.nmem = nmem;
  pl.g.ascal = ascal ? 1 : 0;
  // staging units per thread: the widest slice's slab
  const int64_t units = 8 * (pl.g.Msl / cw + (nmem < pl.g.Nb ? nmem : pl.g.Nb) / cw);
  pl.upt = (int)ceil_div(units, WR_NT);
  if (pl.upt > WR_MAXU) return false;
  pl.lds = (size_t)2 * (pl.g.Ma + pl.g.Nb) * WR_LDK * sizeof(uint16_t);
  if (pl.lds > 160 * 1024) return false;
  int64_t S = target / pl.slices;
  if (S < 1) S = 1;
  if (S > smax) S = smax;
  pl.g.steps_per = ceil_div(steps, S);
  pl.S = ceil_div(steps, pl.g.steps_per);
  // per call (tests compare both orders).  Off by default: isolated the s2conv gather 192 -> 184 us and a 5-slice
  // linear product 33.2 -> 31.9 us, but the step 2374 / 2378 -> 2366 / 2369 utt/s (profiles/r06/r6aj/); KDFM_WGR_XGRP=1
  pl.g.xgrp = (pl.slices > 1 && pl.mslices == 1 && env_i("KDFM_WGR_XGRP", 0)) ? 1 : 0;
  return true;
}

template <int MBW, int NBW, bool CONV, int BIN = 0, bool C2D = false>
int wr_launch(const GemmP& p, const WrPlan& pl, hipStream_t st) {
  static const int pd = env_i("KDFM_WGR_PD", 2);
  auto go = [&](auto kern) {
    static bool once = [&] {
      return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==
             hipSuccess;
    }();
    (void)once;
    hipLaunchKernelGGL(kern, dim3((unsigned)(pl.S * (p.A2 ? 2 : 1)), (unsigned)pl.slices, (unsigned)pl.mslices),
                       dim3(WR_NT), pl.lds, st, p, pl.g);
  };
  if (pl.upt <= 1) {
    if (pd >= 2) go(wgr_kernel<MBW, NBW, CONV, 2, 1, BIN, C2D>); else go(wgr_kernel<MBW, NBW, CONV, 1, 1, BIN, C2D>);
  } else {
    // two slabs of two units each next to an 18-block accumulator tile exceed the 256 registers of
    // a 2-waves-per-SIMD wave (spills): one slab in flight there
    if (pd >= 2 && MBW * NBW < 18) go(wgr_kernel<MBW, NBW, CONV, 2, 2, BIN, C2D>);
    else go(wgr_kernel<MBW, NBW, CONV, 1, 2, BIN, C2D>);
  }
  return check_launch("kdfm_gemm(wgrad rows)");
}

}  // namespace

// per-XCD slot accumulation (GemmP::xslots) for the register-staged kernel: non-deterministic mode
// only (float atomics), and only where it saves traffic (>= 16 splits: 8 slots + a memset instead of
// S raw partials written and read back).  OFF by default (KDFM_WGR_XCD=1 enables it): in the step the
// slot atomics + memset made the weight-gradient stream slower, not faster -- 2051 utt/s with the
// per-split partials vs 1826 with the slots, same box, interleaved (profiles/r04/r4c_bench_*.log).
constexpr int WR_XSLOTS = 8;
bool wr_use_xslots(const WrPlan& pl) {
  const int on = env_i("KDFM_WGR_XCD", 0);   // read per call, like KDFM_WGR_MSL (tests compare both)
  return on && !deterministic() && !pl.dma && pl.S >= 2 * WR_XSLOTS;
}

// zero the slots (stream-ordered) and mark the launch parameters
int wr_prep_xslots(GemmP& q, const WrPlan& pl, hipStream_t st) {
  if (q.A2 || !wr_use_xslots(pl)) return 0;   // paired launches keep the per-split partials
  q.xslots = WR_XSLOTS;
  if (hipMemsetAsync(q.ws, 0, sizeof(float) * WR_XSLOTS * q.M * q.N, st) != hipSuccess)
    return check_launch("kdfm wgrad rows (slot memset)");
  return 0;
}

int wr_fold(const GemmP& p, int64_t S, hipStream_t st) {
  fold_launch<false>(p, p.xslots ? (int64_t)p.xslots : S, st);
  return check_launch("kdfm wgrad rows (fold)");
}

int64_t wgrad_rows_ws(const GemmP& p, int amode, int bmode, int64_t batch) {
  GemmP q = p;
  q.A = reinterpret_cast<const float*>(16);  // alignment checks only
  q.B = reinterpret_cast<const float*>(16);
  WrPlan pl;
  if (!wr_plan(q, amode, bmode, batch, pl)) return 0;
  return pl.S * p.M * p.N;
}

int try_wgrad_rows(const GemmP& p, int amode, int bmode, int64_t batch, hipStream_t st) {
  WrPlan pl;
  if (!p.ws || !wr_plan(p, amode, bmode, batch, pl)) return -1;
  if (p.ws_len < pl.S * p.M * p.N) return -1;
  GemmP q = p;
  int rc = wr_prep_xslots(q, pl, st);
  if (rc) return rc;
  const int key = pl.w.mbw * 10 + pl.w.nbw;
  if (bmode == KDFM_LD_CONV) {
    switch (key) {
      case 32: rc = wr_launch<3, 2, true>(q, pl, st); break;
      case 33: rc = wr_launch<3, 3, true>(q, pl, st); break;
      case 34: rc = wr_launch<3, 4, true>(q, pl, st); break;
      case 36: rc = wr_launch<3, 6, true>(q, pl, st); break;
      default: rc = wr_launch<6, 3, true>(q, pl, st); break;
    }
  } else {
    switch (key) {
      case 32: rc = wr_launch<3, 2, false>(q, pl, st); break;
      case 33: rc = wr_launch<3, 3, false>(q, pl, st); break;
      case 34: rc = wr_launch<3, 4, false>(q, pl, st); break;
      case 36: rc = wr_launch<3, 6, false>(q, pl, st); break;
      default: rc = wr_launch<6, 3, false>(q, pl, st); break;
    }
  }
  if (rc) return rc;
  return wr_fold(q, pl.S, st);
}

}  // namespace kdfm

namespace kdfm {
namespace {

// ---- bf16 weight gradient streamed by LDS-DMA -----------------------------------------------------
// Dense bf16 operands dY (rows, M) and X (rows, N) (M, N multiples of 8; no conv taps, no segments):
// every 32-row slab of dY and of X is one contiguous run of HBM, copied into LDS unchanged by
// global_load_lds_dwordx4 (a wave-instruction moves 1 KB; no staging registers, no transpose pass),
// and the MFMA fragments are read TRANSPOSED out of the row-major images with ds_read_b64_tr_b16
// (dW = dY^T X: A = dY^T, B = X, both summing over the slab's rows).  A ring of NS slab buffers keeps
// NS - 2 slabs in flight behind the one being multiplied: every wave issues exactly pw DMA
// instructions per slab (pieces past the image repeat its last piece, slabs past the split's end
// repeat its last slab), so the wait for slab s is the fixed count vmcnt(pw (NS - 2)).  Rows past
// the split's end are loaded from a clamped address and zeroed in LDS before use.  The bias gradient
// (column sums of dY) is one extra MFMA per output-row tile against an all-ones B operand.  Partials
// go out transposed, ws[split][n][m] -- one 16-byte store per accumulator tile -- and
// wgr_fold_kernel<true> adds them in split order (deterministic).
constexpr int WD_NT = 512;

__device__ __forceinline__ void vm_wait(int n) {   // s_waitcnt vmcnt(n) for a wave-uniform n < 64
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(3952); break;
    case 1: __builtin_amdgcn_s_waitcnt(3953); break;
    case 2: __builtin_amdgcn_s_waitcnt(3954); break;
    case 3: __builtin_amdgcn_s_waitcnt(3955); break;
    case 4: __builtin_amdgcn_s_waitcnt(3956); break;
    case 5: __builtin_amdgcn_s_waitcnt(3957); break;
    case 6: __builtin_amdgcn_s_waitcnt(3958); break;
    case 7: __builtin_amdgcn_s_waitcnt(3959); break;
    case 8: __builtin_amdgcn_s_waitcnt(3960); break;
    case 9: __builtin_amdgcn_s_waitcnt(3961); break;
    case 10: __builtin_amdgcn_s_waitcnt(3962); break;
    case 11: __builtin_amdgcn_s_waitcnt(3963); break;
    case 12: __builtin_amdgcn_s_waitcnt(3964); break;
    case 13: __builtin_amdgcn_s_waitcnt(3965); break;
    case 14: __builtin_amdgcn_s_waitcnt(3966); break;
    case 15: __builtin_amdgcn_s_waitcnt(3967); break;
    case 16: __builtin_amdgcn_s_waitcnt(20336); break;
    case 17: __builtin_amdgcn_s_waitcnt(20337); break;
    case 18: __builtin_amdgcn_s_waitcnt(20338); break;
    case 19: __builtin_amdgcn_s_waitcnt(20339); break;
    case 20: __builtin_amdgcn_s_waitcnt(20340); break;
    case 21: __builtin_amdgcn_s_waitcnt(20341); break;
    case 22: __builtin_amdgcn_s_waitcnt(20342); break;
    case 23: __builtin_amdgcn_s_waitcnt(20343); break;
    case 24: __builtin_amdgcn_s_waitcnt(20344); break;
    case 25: __builtin_amdgcn_s_waitcnt(20345); break;
    case 26: __builtin_amdgcn_s_waitcnt(20346); break;
    case 27: __builtin_amdgcn_s_waitcnt(20347); break;
    case 28: __builtin_amdgcn_s_waitcnt(20348); break;
    case 29: __builtin_amdgcn_s_waitcnt(20349); break;
    case 30: __builtin_amdgcn_s_waitcnt(20350); break;
    case 31: __builtin_amdgcn_s_waitcnt(20351); break;
    case 32: __builtin_amdgcn_s_waitcnt(36720); break;
    case 33: __builtin_amdgcn_s_waitcnt(36721); break;
    case 34: __builtin_amdgcn_s_waitcnt(36722); break;
    case 35: __builtin_amdgcn_s_waitcnt(36723); break;
    case 36: __builtin_amdgcn_s_waitcnt(36724); break;
    case 37: __builtin_amdgcn_s_waitcnt(36725); break;
    case 38: __builtin_amdgcn_s_waitcnt(36726); break;
    case 39: __builtin_amdgcn_s_waitcnt(36727); break;
    case 40: __builtin_amdgcn_s_waitcnt(36728); break;
    case 41: __builtin_amdgcn_s_waitcnt(36729); break;
    case 42: __builtin_amdgcn_s_waitcnt(36730); break;
    case 43: __builtin_amdgcn_s_waitcnt(36731); break;
    case 44: __builtin_amdgcn_s_waitcnt(36732); break;
    case 45: __builtin_amdgcn_s_waitcnt(36733); break;
    case 46: __builtin_amdgcn_s_waitcnt(36734); break;
    case 47: __builtin_amdgcn_s_waitcnt(36735); break;
    case 48: __builtin_amdgcn_s_waitcnt(53104); break;
    case 49: __builtin_amdgcn_s_waitcnt(53105); break;
    case 50: __builtin_amdgcn_s_waitcnt(53106); break;
    case 51: __builtin_amdgcn_s_waitcnt(53107); break;
    case 52: __builtin_amdgcn_s_waitcnt(53108); break;
    case 53: __builtin_amdgcn_s_waitcnt(53109); break;
    case 54: __builtin_amdgcn_s_waitcnt(53110); break;
    case 55: __builtin_amdgcn_s_waitcnt(53111); break;
    case 56: __builtin_amdgcn_s_waitcnt(53112); break;
    case 57: __builtin_amdgcn_s_waitcnt(53113); break;
    case 58: __builtin_amdgcn_s_waitcnt(53114); break;
    case 59: __builtin_amdgcn_s_waitcnt(53115); break;
    case 60: __builtin_amdgcn_s_waitcnt(53116); break;
    case 61: __builtin_amdgcn_s_waitcnt(53117); break;
    case 62: __builtin_amdgcn_s_waitcnt(53118); break;
    case 63: __builtin_amdgcn_s_waitcnt(53119); break;
    default: __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8)); break;
  }
}

typedef short wd_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wd_v4s wd_lds_v4s;
typedef __attribute__((address_space(3))) void wd_lds_void;
typedef __attribute__((address_space(1))) void wd_gl_void;

// lane l: X[8 (l >> 4) + e][n0 + (l & 15)], e = 0..7, of a row-major [32][ld] bf16 image (EXEC full).
// The two ds_read_b64_tr_b16 are issued as inline asm: with LDS-DMA in flight the compiler drains it
// (vmcnt(0)) before any LDS read it can see, which would empty the slab ring every iteration.  The
// caller must retire them (wd_lds_wait) before using the fragment.
__device__ __forceinline__ bf16x8 wd_tr_frag(const uint16_t* img, int ld, int n0, int lane) {
  const int li = lane & 15;
  const uint16_t* a = img + (8 * (lane >> 4) + (li >> 2)) * ld + n0 + 4 * (li & 3);
  const uint32_t a0 = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint16_t*)a);
  wd_v4s lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a0 + 8u * (uint32_t)ld));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// lgkmcnt(0) for the asm reads, tied to the fragments so no use of them is scheduled above it
template <int MBW, int NBW>
__device__ __forceinline__ void wd_lds_wait(bf16x8 (&af)[MBW], bf16x8 (&bf)[NBW]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < MBW; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
  for (int j = 0; j < NBW; ++j) asm volatile("" : "+v"(bf[j]));
}

template <int MBW, int NBW, int NS>
__global__ __launch_bounds__(WD_NT) void wgd_kernel(GemmP p, WdGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t wd_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t kb = (int64_t)blockIdx.x * g.steps_per * 32;
  int64_t ke = kb + g.steps_per * 32;
  if (ke > p.K) ke = p.K;
  if (p.k_dev) {
    const int64_t kd = *p.k_dev;
    if (ke > kd) ke = kd;
  }
  const int nsteps = ke > kb ? (int)((ke - kb + 31) / 32) : 0;
  const int M = (int)p.M;
  const int N = (int)(p.ones_col >= 0 ? p.ones_col : p.N);   // X's memory columns
  const bool bias = p.ones_col >= 0;
  const uint16_t* A = reinterpret_cast<const uint16_t*>(p.A);
  const uint16_t* X = reinterpret_cast<const uint16_t*>(p.B);
  const int npc = g.pa + g.pb;

  // DMA of slab s (clamped to the last) into buffer s % NS: exactly g.pw instructions per wave
  auto issue = [&](int s) {
    const int sc = s < nsteps ? s : nsteps - 1;
    const int64_t r0 = kb + 32 * (int64_t)sc;
    const int64_t vr = ke - r0 < 32 ? ke - r0 : 32;   // valid rows of the slab
    const int va = (int)(vr * M * 2), vb = (int)(vr * N * 2);
    uint16_t* buf = wd_lds + (s % NS) * g.slab;
    for (int i = 0; i < g.pw; ++i) {
      int f = wave + 8 * i;
      f = f < npc ? f : npc - 1;
      const bool isa = f < g.pa;
      const int fl = isa ? f : f - g.pa;
      const int byte = 1024 * fl + 16 * lane;
      const int valid = isa ? va : vb;
      const int src_b = byte < valid ? byte : 0;   // clamped: the lane writes its (padded) slot anyway
      const uint16_t* src = isa ? A + r0 * M + src_b / 2 : X + r0 * N + src_b / 2;
      uint16_t* dst = buf + (isa ? 0 : g.aimg) + fl * 512;
      __builtin_amdgcn_global_load_lds((wd_gl_void*)src, (wd_lds_void*)dst, 16, 0, 0);
    }
  };

  const int wr_ = wave / g.wn, wc_ = wave - (wave / g.wn) * g.wn;
  const int mb0 = wr_ * MBW, nb0 = wc_ * NBW;
  f32x4 acc[MBW][NBW], accb[MBW];
#pragma unroll
  for (int i = 0; i < MBW; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;   // bf16(1.0)
  const bool do_bias = bias && wc_ == 0;

  if (nsteps > 0) {
    for (int s = 0; s < NS - 1; ++s) issue(s);
    for (int s = 0; s < nsteps; ++s) {
      vm_wait(g.pw * (NS - 2));                         // slab s has landed (this wave's part)
      __builtin_amdgcn_s_waitcnt((0xF) | (3 << 14) | (7 << 4));   // lgkmcnt(0): reads of slab s - 1 done
      __builtin_amdgcn_s_barrier();
      const uint16_t* buf = wd_lds + (s % NS) * g.slab;
      const int64_t r0 = kb + 32 * (int64_t)s;
      if (ke - r0 < 32) {   // tail slab: zero its rows past the end (both images), then re-sync
        const int vr = (int)(ke - r0);
        uint16_t* wb = wd_lds + (s % NS) * g.slab;
        for (int e = threadIdx.x; e < (32 - vr) * (M + N); e += WD_NT) {
          const int ea = (32 - vr) * M;
          if (e < ea) wb[vr * M + e] = 0;
          else wb[g.aimg + vr * N + (e - ea)] = 0;
        }
        __syncthreads();
      }
      bf16x8 af[MBW], bfr[NBW];
#pragma unroll
      for (int i = 0; i < MBW; ++i) {
        const int mt = mb0 + i < g.Mt ? mb0 + i : g.Mt - 1;
        af[i] = wd_tr_frag(buf, M, 16 * mt, lane);
      }
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        const int nt = nb0 + j < g.Nt ? nb0 + j : g.Nt - 1;
        bfr[j] = wd_tr_frag(buf + g.aimg, N, 16 * nt, lane);
      }
      issue(s + NS - 1);   // into the buffer of slab s - 1, which every wave has finished reading
      wd_lds_wait<MBW, NBW>(af, bfr);
#pragma unroll
      for (int i = 0; i < MBW; ++i) {
#pragma unroll
        for (int j = 0; j < NBW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if (do_bias) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, accb[i], 0, 0, 0);
      }
    }
    vm_wait(0);   // no LDS-DMA may outlive the workgroup's LDS allocation
  }

  // raw partial of this split, transposed: ws[split][n][m] (n = N: the bias column)
  const int64_t MN = p.M * p.N;
  float* wsp = p.ws + (int64_t)blockIdx.x * MN;
#pragma unroll
  for (int i = 0; i < MBW; ++i) {
    const int m = 16 * (mb0 + i) + 4 * (lane >> 4);
    const bool mok = mb0 + i < g.Mt && m < M;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int n = 16 * (nb0 + j) + (lane & 15);
      if (mok && nb0 + j < g.Nt && n < N)
        *reinterpret_cast<f32x4*>(wsp + (int64_t)n * M + m) = acc[i][j];
    }
    if (do_bias && mok && (lane & 15) == 0) *reinterpret_cast<f32x4*>(wsp + (int64_t)N * M + m) = accb[i];
  }
}

template <int MBW, int NBW>
int wd_launch(const GemmP& p, const WrPlan& pl, hipStream_t st) {
  auto go = [&](auto kern) {
    static bool once = [&] {
      return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==
             hipSuccess;
    }();
    (void)once;
    hipLaunchKernelGGL(kern, dim3((unsigned)pl.S), dim3(WD_NT), pl.lds, st, p, pl.wd);
  };
  if (pl.ns == 8) go(wgd_kernel<MBW, NBW, 8>);
  else go(wgd_kernel<MBW, NBW, 4>);
  return check_launch("kdfm_wgrad_bf16(dma)");
}

int wd_dispatch(const GemmP& p, const WrPlan& pl, hipStream_t st) {
  switch (pl.w.mbw * 10 + pl.w.nbw) {
    case 32: return wd_launch<3, 2>(p, pl, st);
    case 33: return wd_launch<3, 3>(p, pl, st);
    case 34: return wd_launch<3, 4>(p, pl, st);
    case 36: return wd_launch<3, 6>(p, pl, st);
    default: return wd_launch<6, 3>(p, pl, st);
  }
}

// the wgd route: dense bf16 operands, no conv taps / segments, one column slice, slabs that fit 4 or 8
// buffers in LDS, and long reductions (>= KDFM_WGD_MIN_ROWS rows, default 65,536: the KD heads' stacked
// rows).  LDS-DMA moves ~25-90 GB/s per CU, so a short product (the 12,832-row Conformer layers) spread
// over 31 workgroups took longer than the register-staged kernel over 81 (FFN W1 29 vs 23 us,
// profiles/r03/r3t_wgrad_probe_*.log) while the 1.64M-row FM dW2 over 256 went 228 -> 201 us.
// S: splits of >= KDFM_WGD_STEPS (12) slabs each, at most 256 (one per CU)
bool wd_plan(const GemmP& p, int bmode, WrPlan& pl) {
  static const int on = env_i("KDFM_WGD", 1);
  static const int min_steps = env_i("KDFM_WGD_STEPS", 12);
  static const int64_t min_rows = env_i("KDFM_WGD_MIN_ROWS", 65536);
  if (!on || bmode != KDFM_LD_XC || p.nseg > 1 || p.epi != KDFM_EPI_ATOMIC || p.K < min_rows) return false;
  const int64_t nmem = p.ones_col >= 0 ? p.ones_col : p.N;
  if (p.ones_col >= 0 && p.ones_col != p.N - 1) return false;
  if (p.M % 8 || nmem % 8 || p.sAm != 1 || p.sBn != 1 || p.sAk != p.M || p.sBk != nmem) return false;
  if ((((uintptr_t)p.A) | ((uintptr_t)p.B)) & 15) return false;
  if (p.K * (p.M > nmem ? p.M : nmem) * 2 > (int64_t)INT32_MAX * 64) return false;
  const int64_t Mt = ceil_div(p.M, 16), Nt = ceil_div(nmem, 16);
  if (Nt > 24 || !wr_pick(p.M, nmem, pl.w)) return false;
  WdGeo& g = pl.wd;
  g.wm = pl.w.wm;
  g.wn = pl.w.wn;
  g.Mt = (int)Mt;
  g.Nt = (int)Nt;
  g.pa = (int)ceil_div(64 * p.M, 1024);
  g.pb = (int)ceil_div(64 * nmem, 1024);
  g.pw = (int)ceil_div(g.pa + g.pb, WD_NT / 64);
  g.aimg = g.pa * 512;
  g.slab = (g.pa + g.pb) * 512;
  const size_t slab_bytes = (size_t)g.slab * 2;
  pl.ns = slab_bytes * 8 + 64 <= 150 * 1024 ? 8 : (slab_bytes * 4 + 64 <= 150 * 1024 ? 4 : 0);
  if (!pl.ns || g.pw * (pl.ns - 2) > 63) return false;
  pl.lds = slab_bytes * pl.ns + 64;   // + the last buffer's transposed-read overreach
  const int64_t steps = ceil_div(p.K, 32);
  int64_t S = steps / min_steps;
  if (S > 256) S = 256;
  if (S < 1) S = 1;
  g.steps_per = ceil_div(steps, S);
  pl.S = ceil_div(steps, g.steps_per);
  pl.slices = pl.mslices = 1;
  pl.upt = 1;
  pl.bin = 2;
  pl.dma = true;
  return true;
}

}  // namespace
}  // namespace kdfm

// ---- bf16-operand weight gradient (the fused KD-head chains' saved operands) ---------------------
namespace kdfm {
namespace {
template <int BIN>
int wr_dispatch(const GemmP& p, const WrPlan& pl, int bmode, hipStream_t st) {
  const int key = pl.w.mbw * 10 + pl.w.nbw;
  if constexpr (BIN == 2) {
    if (bmode == WR_LD_C2D) {
      switch (key) {
        case 32: return wr_launch<3, 2, false, 2, true>(p, pl, st);
        case 33: return wr_launch<3, 3, false, 2, true>(p, pl, st);
        case 34: return wr_launch<3, 4, false, 2, true>(p, pl, st);
        case 36: return wr_launch<3, 6, false, 2, true>(p, pl, st);
        default: return wr_launch<6, 3, false, 2, true>(p, pl, st);
      }
    }
  }
  if (bmode == KDFM_LD_CONV) {
    switch (key) {
      case 32: return wr_launch<3, 2, true, BIN>(p, pl, st);
      case 33: return wr_launch<3, 3, true, BIN>(p, pl, st);
      case 34: return wr_launch<3, 4, true, BIN>(p, pl, st);
      case 36: return wr_launch<3, 6, true, BIN>(p, pl, st);
      default: return wr_launch<6, 3, true, BIN>(p, pl, st);
    }
  }
  switch (key) {
    case 32: return wr_launch<3, 2, false, BIN>(p, pl, st);
    case 33: return wr_launch<3, 3, false, BIN>(p, pl, st);
    case 34: return wr_launch<3, 4, false, BIN>(p, pl, st);
    case 36: return wr_launch<3, 6, false, BIN>(p, pl, st);
    default: return wr_launch<6, 3, false, BIN>(p, pl, st);
  }
}

GemmP wgrad_bf16_params(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                        int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len) {
  GemmP p{};
  p.A = reinterpret_cast<const float*>(dY);
  p.B = reinterpret_cast<const float*>(X);
  p.C = dW;
  p.M = M;
  p.N = db ? N + 1 : N;
  p.K = rows;
  p.sAm = 1;
  p.sAk = M;
  p.sBk = N;
  p.sBn = 1;
  p.sCm = ldc;
  p.sCn = 1;
  p.alpha = alpha;
  p.epi = KDFM_EPI_ATOMIC;
  p.ones_out = db;
  p.ones_col = db ? N : -1;
  p.ws = ws;
  p.ws_len = ws_len;
  p.splitk = 1;
  return p;
}

// CONV mode: X is (rows, C) frames; column n = tap * C + c reads frame r + tap - pad of the same
// utterance of T frames (zero outside)
void conv_geometry(GemmP& p, int64_t C, int taps, int pad, int64_t T) {
  p.sBk = C;
  p.conv_c = C;
  p.taps = taps;
  p.pad = pad;
  p.conv_t = T;
}

// ---- deferred folds: per-stream arena and job queue (host side) ----
struct DeferState {
  float* arena = nullptr;
  int64_t len = 0, used = 0;
  // since the arena was set: products that did not fit and folded at once (fallbacks), and the largest
  // arena the queue between two flushes would have needed (demand: what a caller sizes the arena from)
  int64_t want = 0, fallbacks = 0, peak_want = 0;
  std::vector<FoldJob> jobs;
};
std::mutex g_defer_mu;
std::unordered_map<void*, DeferState>& defer_map() {
  static std::unordered_map<void*, DeferState> m;
  return m;
}

// n floats of the stream's fold arena (16-byte aligned), or null when the stream does not defer / it is full
float* defer_reserve(hipStream_t st, int64_t n) {
  std::lock_guard<std::mutex> g(g_defer_mu);
  auto it = defer_map().find((void*)st);
  if (it == defer_map().end() || !it->second.arena) return nullptr;
  DeferState& d = it->second;
  const int64_t need = (n + 3) / 4 * 4;
  d.want += need;
  if (d.want > d.peak_want) d.peak_want = d.want;
  if (d.used + need > d.len) {
    ++d.fallbacks;
    return nullptr;
  }
  float* r = d.arena + d.used;
  d.used += need;
  return r;
}

void defer_push(hipStream_t st, const GemmP& p, const float* ws, float* C, float* ones, int64_t S, bool trans) {
  FoldJob j;
  j.ws = ws; j.C = C; j.ones = ones;
  j.M = p.M; j.N = p.N; j.sCm = p.sCm; j.sCn = p.sCn; j.ones_col = p.ones_col; j.S = S;
  j.alpha = p.alpha; j.trans = trans ? 1 : 0;
  std::lock_guard<std::mutex> g(g_defer_mu);
  defer_map()[(void*)st].jobs.push_back(j);
}

// the 4-wide fold applies (and the product keeps per-split partials)
bool defer_ok(const GemmP& p, const WrPlan& pl) { return (p.M * p.N) % 4 == 0 && !wr_use_xslots(pl); }

int wgrad_bf16_run(const GemmP& p, int bmode, hipStream_t st) {
  WrPlan pl;
  KDFM_REQUIRE(wr_plan(p, KDFM_LD_XC, bmode, 1, pl, true, true), "shape not supported by the row-parallel kernel");
  KDFM_REQUIRE(p.ws_len >= pl.S * p.M * p.N, "workspace too small (kdfm_wgrad_bf16*_ws)");
  set_route(ROUTE_WGRAD_ROWS);
  // deferred fold: the partials go to the stream's arena and the fold joins the next kdfm_wgrad_fold_flush
  float* dws = defer_ok(p, pl) ? defer_reserve(st, pl.S * p.M * p.N) : nullptr;
  if (dws) {
    GemmP q = p;
    q.ws = dws;
    const int rc = pl.dma ? wd_dispatch(q, pl, st)
                          : (pl.bin == 2 ? wr_dispatch<2>(q, pl, bmode, st) : wr_dispatch<1>(q, pl, bmode, st));
    if (rc) return rc;
    defer_push(st, q, dws, q.C, q.ones_out, pl.S, pl.dma);
    return KDFM_OK;
  }
  if (pl.dma) {
    const int rc = wd_dispatch(p, pl, st);
    if (rc) return rc;
    fold_launch<true>(p, pl.S, st);
    return check_launch("kdfm_wgrad_bf16(fold)");
  }
  GemmP q = p;
  int rc = wr_prep_xslots(q, pl, st);
  if (rc) return rc;
  rc = pl.bin == 2 ? wr_dispatch<2>(q, pl, bmode, st) : wr_dispatch<1>(q, pl, bmode, st);
  if (rc) return rc;
  return wr_fold(q, pl.S, st);
}
}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_wgrad_bf16_ws(int64_t rows, int64_t M, int64_t N, int32_t bias) {
  using namespace kdfm;
  GemmP p = wgrad_bf16_params(reinterpret_cast<const uint16_t*>(16), reinterpret_cast<const uint16_t*>(16), nullptr, N,
                              bias ? reinterpret_cast<float*>(16) : nullptr, rows, M, N, 1.f, nullptr, 0);
  WrPlan pl;
  if (!wr_plan(p, KDFM_LD_XC, KDFM_LD_XC, 1, pl, true, true)) return -1;
  return pl.S * p.M * p.N;
}

int kdfm_wgrad_bf16(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                    int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dY && X && dW && ws, "null pointer");
  KDFM_REQUIRE(rows > 0 && M > 0 && N > 0 && M % 4 == 0 && N % 4 == 0, "M, N must be positive multiples of 4");
  KDFM_REQUIRE(((((uintptr_t)dY) | ((uintptr_t)X)) & 15) == 0, "operands must be 16-byte aligned");
  KDFM_REQUIRE(ldc >= N, "ldc < N");
  GemmP p = wgrad_bf16_params(dY, X, dW, ldc, db, rows, M, N, alpha, ws, ws_len);
  return wgrad_bf16_run(p, KDFM_LD_XC, as_stream(stream));
}

int64_t kdfm_wgrad_bf16_s2conv_ws(int64_t B, int64_t T1, int64_t F1, int64_t C) {
  using namespace kdfm;
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  GemmP p = wgrad_bf16_params(reinterpret_cast<const uint16_t*>(16), reinterpret_cast<const uint16_t*>(16), nullptr,
                              9 * C, reinterpret_cast<float*>(16), B * T2 * F2, C, 9 * C, 1.f, nullptr, 0);
  p.conv_c = C;
  p.c2_T1 = T1;
  p.c2_F1 = F1;
  p.c2_T2 = T2;
  p.c2_F2 = F2;
  WrPlan pl;
  if (!wr_plan(p, KDFM_LD_XC, WR_LD_C2D, 1, pl, true, true)) return -1;
  return pl.S * p.M * p.N;
}

int kdfm_wgrad_bf16_s2conv(const uint16_t* dY, const uint16_t* X, int64_t ldx, const int64_t* len_in, float* dW,
                           float* db, int64_t B, int64_t T1, int64_t F1, int64_t C, float alpha, float* ws,
                           int64_t ws_len, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dY && X && dW && db && ws, "null pointer");
  KDFM_REQUIRE(B > 0 && T1 > 0 && F1 >= 7 && C > 0 && C % 8 == 0, "B, T1 > 0, F1 >= 7, C a positive multiple of 8");
  KDFM_REQUIRE(ldx >= C && ldx % 8 == 0, "ldx must be a multiple of 8, >= C");
  KDFM_REQUIRE(((((uintptr_t)dY) | ((uintptr_t)X)) & 15) == 0, "operands must be 16-byte aligned");
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  GemmP p = wgrad_bf16_params(dY, X, dW, 9 * C, db, B * T2 * F2, C, 9 * C, alpha, ws, ws_len);
  p.conv_c = C;
  p.c2_T1 = T1;
  p.c2_F1 = F1;
  p.c2_T2 = T2;
  p.c2_F2 = F2;
  p.c2_len = len_in;
  p.c2_ld = ldx;
  return wgrad_bf16_run(p, WR_LD_C2D, as_stream(stream));
}

int kdfm_wgrad_bf16_pair(const uint16_t* dY, const uint16_t* X, float* dW, float* db, const uint16_t* dY2,
                         const uint16_t* X2, float* dW2, float* db2, int64_t ldc, int64_t rows, int64_t M, int64_t N,
                         float alpha, float* ws, int64_t ws_len, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dY && X && dW && dY2 && X2 && dW2 && ws, "null pointer");
  KDFM_REQUIRE((db == nullptr) == (db2 == nullptr), "both products have a bias gradient or neither");
  KDFM_REQUIRE(rows > 0 && M > 0 && N > 0 && M % 4 == 0 && N % 4 == 0, "M, N must be positive multiples of 4");
  KDFM_REQUIRE(((((uintptr_t)dY) | ((uintptr_t)X) | ((uintptr_t)dY2) | ((uintptr_t)X2)) & 15) == 0,
               "operands must be 16-byte aligned");
  KDFM_REQUIRE(ldc >= N, "ldc < N");
  const int64_t one = kdfm_wgrad_bf16_ws(rows, M, N, db ? 1 : 0);
  KDFM_REQUIRE(one > 0 && ws_len >= 2 * one, "workspace too small (2 x kdfm_wgrad_bf16_ws)");
  hipStream_t st = as_stream(stream);
  GemmP p = wgrad_bf16_params(dY, X, dW, ldc, db, rows, M, N, alpha, ws, one);
  WrPlan pl;
  KDFM_REQUIRE(wr_plan(p, KDFM_LD_XC, KDFM_LD_XC, 1, pl, true, true), "shape not supported by the row-parallel kernel");
  if (pl.dma) {   // long reductions take the LDS-DMA kernel: two ordinary launches
    int rc = wgrad_bf16_run(p, KDFM_LD_XC, st);
    if (rc) return rc;
    GemmP q = wgrad_bf16_params(dY2, X2, dW2, ldc, db2, rows, M, N, alpha, ws + one, one);
    return wgrad_bf16_run(q, KDFM_LD_XC, st);
  }
  // one grid of 2 S workgroups (blocks [S, 2 S) run the second product), one fold launch over both:
  // each product's splits, partial layout and fold order are those of a single launch (bitwise equal)
  p.A2 = reinterpret_cast<const float*>(dY2);
  p.B2 = reinterpret_cast<const float*>(X2);
  p.C2 = dW2;
  p.ones_out2 = db2;
  p.ws2 = ws + one;
  set_route(ROUTE_WGRAD_ROWS);
  const int64_t oner = (one + 3) / 4 * 4;
  float* dws = defer_ok(p, pl) ? defer_reserve(st, 2 * oner) : nullptr;
  if (dws) {   // deferred folds (both products' partials in the stream's arena)
    p.ws = dws;
    p.ws2 = dws + oner;
  }
  const int rc = pl.bin == 2 ? wr_dispatch<2>(p, pl, KDFM_LD_XC, st) : wr_dispatch<1>(p, pl, KDFM_LD_XC, st);
  if (rc) return rc;
  if (dws) {
    defer_push(st, p, p.ws, p.C, p.ones_out, pl.S, false);
    defer_push(st, p, p.ws2, p.C2, p.ones_out2, pl.S, false);
    return KDFM_OK;
  }
  return wr_fold(p, pl.S, st);
}

int kdfm_wgrad_bf16_dev(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                        const int64_t* rows_dev, int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len,
                        void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(rows_dev, "rows_dev is required (kdfm_wgrad_bf16 for a host row count)");
  KDFM_REQUIRE(dY && X && dW && ws, "null pointer");
  KDFM_REQUIRE(rows > 0 && M > 0 && N > 0 && M % 4 == 0 && N % 4 == 0, "M, N must be positive multiples of 4");
  KDFM_REQUIRE(ldc >= N, "ldc < N");
  KDFM_REQUIRE(ws_len >= kdfm_wgrad_bf16_ws(rows, M, N, db ? 1 : 0), "workspace too small (kdfm_wgrad_bf16_ws)");
  GemmP p = wgrad_bf16_params(dY, X, dW, ldc, db, rows, M, N, alpha, ws, ws_len);
  p.k_dev = rows_dev;
  return wgrad_bf16_run(p, KDFM_LD_XC, as_stream(stream));
}

int64_t kdfm_wgrad_bf16_seg_ws(int64_t rows, int64_t M, int64_t N, int64_t seg_rows) {
  using namespace kdfm;
  // the launch's own preconditions (kdfm_wgrad_bf16_seg): a query must never accept a shape the
  // launch rejects (with one segment wr_plan would not check seg_rows % 32 itself)
  if (seg_rows <= 0 || seg_rows % 32 || rows % seg_rows || rows / seg_rows > 16 || M % 4 || N % 4) return -1;
  GemmP p = wgrad_bf16_params(reinterpret_cast<const uint16_t*>(16), reinterpret_cast<const uint16_t*>(16), nullptr, N,
                              nullptr, rows, M, N, 1.f, nullptr, 0);
  p.nseg = (int)(rows / seg_rows);
  p.seg_rows = seg_rows;
  p.N = N + p.nseg;
  p.ones_col = N;
  p.ones_out = reinterpret_cast<float*>(16);
  WrPlan pl;
  if (!wr_plan(p, KDFM_LD_XC, KDFM_LD_XC, 1, pl, true, true)) return -1;
  return pl.S * p.M * p.N;
}

int kdfm_wgrad_bf16_seg(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t seg_rows,
                        int64_t rows, int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dY && X && dW && db && ws, "null pointer");
  KDFM_REQUIRE(rows > 0 && M > 0 && N > 0 && M % 4 == 0 && N % 4 == 0, "M, N must be positive multiples of 4");
  KDFM_REQUIRE(seg_rows > 0 && seg_rows % 32 == 0 && rows % seg_rows == 0 && rows / seg_rows <= 16,
               "seg_rows must be a multiple of 32 dividing rows into at most 16 segments");
  KDFM_REQUIRE(((((uintptr_t)dY) | ((uintptr_t)X)) & 15) == 0, "operands must be 16-byte aligned");
  KDFM_REQUIRE(ldc >= N, "ldc < N");
  GemmP p = wgrad_bf16_params(dY, X, dW, ldc, nullptr, rows, M, N, alpha, ws, ws_len);
  p.nseg = (int)(rows / seg_rows);
  p.seg_rows = seg_rows;
  p.N = N + p.nseg;
  p.ones_col = N;
  p.ones_out = db;
  return wgrad_bf16_run(p, KDFM_LD_XC, as_stream(stream));
}

int64_t kdfm_wgrad_bf16_conv_ws(int64_t rows, int64_t M, int64_t C, int32_t taps, int32_t pad, int64_t T, int32_t bias) {
  using namespace kdfm;
  GemmP p = wgrad_bf16_params(reinterpret_cast<const uint16_t*>(16), reinterpret_cast<const uint16_t*>(16), nullptr,
                              taps * C, bias ? reinterpret_cast<float*>(16) : nullptr, rows, M, taps * C, 1.f, nullptr, 0);
  conv_geometry(p, C, taps, pad, T);
  WrPlan pl;
  if (!wr_plan(p, KDFM_LD_XC, KDFM_LD_CONV, 1, pl, true, true)) return -1;
  return pl.S * p.M * p.N;
}

int kdfm_wgrad_bf16_conv(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                         int64_t M, int64_t C, int32_t taps, int32_t pad, int64_t T, float alpha, float* ws,
                         int64_t ws_len, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dY && X && dW && ws, "null pointer");
  KDFM_REQUIRE(rows > 0 && M > 0 && C > 0 && M % 4 == 0 && C % 4 == 0, "M, C must be positive multiples of 4");
  KDFM_REQUIRE(taps >= 1 && pad >= 0 && pad < taps && T >= 1 && rows % T == 0, "bad conv geometry");
  KDFM_REQUIRE(((((uintptr_t)dY) | ((uintptr_t)X)) & 15) == 0, "operands must be 16-byte aligned");
  KDFM_REQUIRE(ldc >= taps * C, "ldc < taps * C");
  GemmP p = wgrad_bf16_params(dY, X, dW, ldc, db, rows, M, taps * C, alpha, ws, ws_len);
  conv_geometry(p, C, taps, pad, T);
  return wgrad_bf16_run(p, KDFM_LD_CONV, as_stream(stream));
}

int kdfm_wgrad_set_fold_arena(void* stream, float* arena, int64_t len) {
  using namespace kdfm;
  KDFM_REQUIRE(!arena || (len > 0 && ((uintptr_t)arena & 15) == 0), "arena must be 16-byte aligned with len > 0");
  std::lock_guard<std::mutex> g(g_defer_mu);
  DeferState& d = defer_map()[stream];
  KDFM_REQUIRE(d.jobs.empty(), "folds still queued on this stream: kdfm_wgrad_fold_flush first");
  d.arena = arena;
  d.len = arena ? len : 0;
  d.used = 0;
  d.want = d.fallbacks = d.peak_want = 0;
  return KDFM_OK;
}

int kdfm_wgrad_fold_stats(void* stream, int64_t* out3) {
  using namespace kdfm;
  KDFM_REQUIRE(out3 != nullptr, "null output");
  std::lock_guard<std::mutex> g(g_defer_mu);
  auto it = defer_map().find(stream);
  out3[0] = out3[1] = out3[2] = 0;
  if (it == defer_map().end()) return KDFM_OK;
  out3[0] = (int64_t)it->second.jobs.size();
  out3[1] = it->second.fallbacks;
  out3[2] = it->second.peak_want;
  return KDFM_OK;
}

int kdfm_wgrad_fold_discard_all(void) {
  using namespace kdfm;
  std::lock_guard<std::mutex> g(g_defer_mu);
  int n = 0;
  for (auto& kv : defer_map()) {
    n += (int)kv.second.jobs.size();
    kv.second = DeferState{};
  }
  return n;
}

int kdfm_wgrad_fold_flush(void* stream) {
  using namespace kdfm;
  std::vector<FoldJob> jobs;
  {
    std::lock_guard<std::mutex> g(g_defer_mu);
    auto it = defer_map().find(stream);
    if (it == defer_map().end()) return KDFM_OK;
    jobs.swap(it->second.jobs);
    it->second.used = 0;   // the stream's next products reuse the arena after these folds (stream order)
    it->second.want = 0;
  }
  hipStream_t st = as_stream(stream);
  // the byte ranges a job's fold writes (its gradient block, its bias row(s)): jobs in one launch run
  // concurrently, so a job adding into memory an earlier queued job also adds into (two products into one
  // gradient: the heads' layer halves, per-step products) starts a new launch -- stream order keeps the
  // queue's order for them
  auto ranges = [](const FoldJob& j, uintptr_t (&r)[2][2]) {
    const int64_t nmem = j.ones_col >= 0 ? j.ones_col : j.N;
    r[0][0] = (uintptr_t)j.C;
    r[0][1] = (uintptr_t)(j.C + (j.M - 1) * j.sCm + (nmem - 1) * j.sCn) + sizeof(float);
    r[1][0] = r[1][1] = 0;
    if (j.ones_col >= 0 && j.ones) {
      r[1][0] = (uintptr_t)j.ones;
      r[1][1] = (uintptr_t)(j.ones + (j.N - j.ones_col) * j.M);
    }
  };
  auto overlap = [](const uintptr_t (&a)[2][2], const uintptr_t (&b)[2][2]) {
    for (int x = 0; x < 2; ++x)
      for (int y = 0; y < 2; ++y)
        if (a[x][1] > a[x][0] && b[y][1] > b[y][0] && a[x][0] < b[y][1] && b[y][0] < a[x][1]) return true;
    return false;
  };
  FoldBatch fb{};
  uintptr_t rg[FB_MAXJ][2][2];
  auto launch = [&]() -> int {
    if (fb.n == 0) return KDFM_OK;
    hipLaunchKernelGGL(wgr_fold_batch_kernel, dim3((unsigned)fb.blk0[fb.n]), dim3(64 * WF_WAVES), 0, st, fb);
    fb.n = 0;
    fb.blk0[0] = 0;
    return check_launch("kdfm_wgrad_fold_flush");
  };
  fb.blk0[0] = 0;
  for (const FoldJob& job : jobs) {
    uintptr_t r[2][2];
    ranges(job, r);
    bool clash = fb.n == FB_MAXJ;
    for (int k = 0; k < fb.n && !clash; ++k) clash = overlap(r, rg[k]);
    if (clash) {
      const int rc = launch();
      if (rc) return rc;
    }
    fb.j[fb.n] = job;
    for (int x = 0; x < 2; ++x)
      for (int y = 0; y < 2; ++y) rg[fb.n][x][y] = r[x][y];
    fb.blk0[fb.n + 1] = fb.blk0[fb.n] + ceil_div(job.M * job.N, 256);
    ++fb.n;
  }
  return launch();
}

int64_t kdfm_wgrad_fold_pending(void* stream) {
  using namespace kdfm;
  std::lock_guard<std::mutex> g(g_defer_mu);
  auto it = defer_map().find(stream);
  return it == defer_map().end() ? 0 : (int64_t)it->second.jobs.size();
}

}  // extern "C"
