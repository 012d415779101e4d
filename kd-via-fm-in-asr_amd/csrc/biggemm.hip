// Large-tile bf16 GEMM for the wide layer products (d_model >= 512: Conformer-large, FastConformer /
// FastConformer-XL -- BASELINE.json configs[3] / [4]; fast-conformer_ctc_bpe.yaml:29 XLarge d=1024), where no
// fused LN-block kernel applies and the products are large and MFMA-friendly (M = B*T' >= 4k rows, N, K >= 512).
//
// C[m][n] = epi(alpha * sum_k A(m, k) B(k, n)) with bf16 operands in HBM and f32 accumulation:
//   * each operand is either K-CONTIGUOUS (A stored [m][k], B stored [n][k]: the forward's x W^T) or
//     K-MAJOR (A stored [k][m], B stored [k][n]: the data gradient's W, the weight gradient's dY and X) --
//     three instantiations cover every Linear: forward (A, B k-contiguous), data gradient (A k-contiguous,
//     B = W k-major), weight gradient (both k-major, the reduction over rows);
//   * workgroup tile BM x BN (256x256 / 256x128 / 128x128, picked per shape to fill the 256 CUs), 8 or 4 waves,
//     each wave a (BM/WM) x (BN/WN) block of v_mfma_f32_16x16x32_bf16 tiles, K step 64;
//   * operand tiles staged HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: one wave-instruction moves 1 KB, no
//     staging registers), two LDS stages, the next stage's DMA in flight while the current one's MFMAs run, one
//     barrier per K step; the k-contiguous images are [row][64 k] with 128-byte rows whose 16-byte chunks are
//     XOR-swizzled by (row >> 1) & 7 (conflict-free ds_read_b128 fragment reads), the k-major images are
//     [64 k][cols] rows whose 8-byte units are XOR-swizzled by the row's (bits 0-1, bit 3) -- the fragments are
//     read TRANSPOSED with ds_read_b64_tr_b16 (conflict-free); the swizzle is applied to the DMA's per-lane
//     SOURCE address (the LDS destination of an LDS-DMA is lane-linear);
//   * the fused epilogue is gemm_common.h's (bias, SiLU, ReLU, dropout, STORE_PRE, dReLU / dSiLU, residual,
//     BETA, row mask: the same per-element semantics as every other kdfm_gemm route), f32 or bf16 output
//     (a bf16 output is what the next product reads), or the weight-gradient accumulate C += alpha * acc with
//     the bias gradient (row sums of A) from one extra MFMA per row tile against an all-ones operand.
// Deterministic: every output element has one writer and a fixed summation order (no split-K, no atomics).
#include "gemm_common.h"

#include <cstdlib>

namespace kdfm {
namespace {

constexpr int BG_BK = 64;
// epilogue modes beyond gemm_common.h's SKC_EPI_*: the weight-gradient accumulate, without / with the bias gradient
// (the extra accumulators of the latter exist only in its instances: they cost 4 * FM registers)
constexpr int BG_ACC = 98, BG_ACCB = 99;
// the data gradient through a dropped-out SiLU (the FFN's linear2 dX: dh = drop(dY W2) * silu'(h)), flags
// KDFM_EPI_DSILU | KDFM_EPI_DROPOUT with the pre-activation as aux: epi_apply's arithmetic in that order
constexpr int BG_DSILU_DROP = 97;

typedef short bg_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void bg_lds_void;
typedef __attribute__((address_space(1))) void bg_gl_void;

struct BigP {
  const uint16_t* A;
  const uint16_t* B;
  int64_t lda, ldb;   // row strides (elements) of the stored operands
  uint16_t* C16;      // bf16 output (row stride g.sCm) instead of g.C when non-null
  float* ones_out;    // ones_out[m] += alpha * sum_k A(m, k) (accumulate mode)
  int accum;          // C[m][n] += alpha * acc
  int tn;             // column tiles
  // split reduction (the weight-gradient layout when its tiles alone cannot fill the chip): split s sums K rows
  // [s kchunk, min(K, (s + 1) kchunk)) into raw partials ws[s][m][n] (bias: wsb[s][m]), folded in split order by
  // big_fold_kernel (deterministic)
  int splits;
  int64_t kchunk;
  float* ws;
  float* wsb;
  // fp8 instance (e4m3 operands, MX block scaling): one e8m0 scale byte per 32 consecutive k of a row, stored
  // stage-major xs[((k / 128) * rows + row) * 4 + (k / 32) % 4] (kdfm_fp8_quant_mx), applied by the MFMA itself
  const uint8_t* xsa;
  const uint8_t* xsb;
  GemmP g;            // M, N, K, C, strides and the epilogue fields
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// 16-byte chunk swizzle of a k-contiguous image row (128 B = 8 chunks)
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 7; }
// 8-byte unit swizzle of a k-major image row: 4 * (row bits 0-1 | bit 3 << 2) (a multiple of 4 units, i.e. of
// 2 chunks, so one 16-byte DMA chunk keeps its two units together)
__device__ __forceinline__ int km_swz8(int row) { return 4 * ((row & 3) | (((row >> 3) & 1) << 2)); }

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// fragment of 16 rows x 32 k out of a k-contiguous [rows][64] image: lane l -> row r0 + (l & 15),
// k = 32 hh + 8 (l >> 4) .. + 7
__device__ __forceinline__ bf16x8 frag_kc(const uint16_t* img, int r0, int hh, int lane) {
  const int r = r0 + (lane & 15);
  const int p = ((lane >> 4) + 4 * hh) ^ kc_swz(r);
  const uint32_t a = lds_addr(img + r * BG_BK + 8 * p);
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

typedef int bg_v8i __attribute__((ext_vector_type(8)));

// fp8 fragment of 16 rows x 128 k out of a k-contiguous [rows][128 bytes] image (the bf16 image's byte layout):
// v_mfma_scale_f32_16x16x128_f8f6f4's operand map, lane l (g = l >> 4) -> row r0 + (l & 15), operand byte j -> k =
// 16 g + j for j < 16 and 64 + 16 g + (j - 16) for j >= 16 (16-byte chunks g and 4 + g of the row); the e8m0 scale
// of row r, 32-k block b is lane r + 16 b's scale byte (tools/fp8_scale_probe.py measured both on gfx950: each
// lane's scale covers 16 bytes in each of two lanes, not its own 32 bytes)
__device__ __forceinline__ bg_v8i frag_kc8(const uint16_t* img, int r0, int lane) {
  const int r = r0 + (lane & 15);
  const int g = lane >> 4;
  const uint32_t a0 = lds_addr(img + r * BG_BK + 8 * (g ^ kc_swz(r)));
  const uint32_t a1 = lds_addr(img + r * BG_BK + 8 * ((4 + g) ^ kc_swz(r)));
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i lo, hi;
  asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(a0));
  asm volatile("ds_read_b128 %0, %1" : "=v"(hi) : "v"(a1));
  return bg_v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// fragment of 16 columns x 32 k out of a k-major [64][W] image: lane l (g = l >> 4, li = l & 15) -> column
// c0 + li, k = 32 hh + 8 g + e (e < 4: first transposed read, rows 32 hh + 8 g + q; e >= 4: rows + 4)
template <int W>
__device__ __forceinline__ bf16x8 frag_km(const uint16_t* img, int c0, int hh, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const int row = 32 * hh + 8 * g + (li >> 2);
  const int u = ((c0 >> 2) + (li & 3)) ^ km_swz8(row);
  const uint32_t a = lds_addr(img + row * W + 4 * u);
  bg_v4s lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a + 8u * (uint32_t)W));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EMODE, bool F8 = false>
__global__ __launch_bounds__(WM* WN * 64) void big_gemm_kernel(BigP p) {
  static_assert(!F8 || (!AT && !BT), "the fp8 instance is k-contiguous only");
  constexpr int KSTEP = F8 ? 2 * BG_BK : BG_BK;   // k per stage: 128-byte image rows either way
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int AIMG = BM * BG_BK, BIMG = BN * BG_BK;   // elements per stage
  // fp8: each stage also holds the A and B scale bytes of its 128 k (4 per row: <= 1 KB each)
  constexpr int STAGE = AIMG + BIMG + (F8 ? 1024 : 0);
  constexpr int PA = BM / 8, PB = BN / 8, PW = (PA + PB) / NW;   // 1 KB DMA pieces: A, B, per wave
  static_assert((PA + PB) % NW == 0, "pieces per wave");
  extern __shared__ __attribute__((aligned(16))) uint16_t bg_lds[];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int64_t blk = xcd_block();   // the splits of one tile are neighbours (one XCD)
  const int64_t tile = blk / p.splits;
  const int sp = (int)(blk - tile * p.splits);
  const int64_t tm = tile / p.tn, tnn = tile % p.tn;
  const int64_t m0 = tm * BM, n0 = tnn * BN;
  const int64_t M = p.g.M, N = p.g.N;
  const int64_t kb = (int64_t)sp * p.kchunk;
  const int64_t K = (kb + p.kchunk < p.g.K) ? kb + p.kchunk : p.g.K;   // this split's end row
  const int nk = K > kb ? (int)((K - kb + KSTEP - 1) / KSTEP) : 0;

  // DMA of K step t into stage buffer s: exactly PW wave-instructions per wave
  auto issue = [&](int t, int s) {
    const int64_t k0 = kb + (int64_t)t * KSTEP;
    uint16_t* buf = bg_lds + s * STAGE;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int f = wave + NW * i;
      const bool isa = f < PA;
      const int fl = isa ? f : f - PA;
      const uint16_t* X = isa ? p.A : p.B;
      const int64_t ld = isa ? p.lda : p.ldb;
      const int64_t R = isa ? M : N, r0 = isa ? m0 : n0;
      const bool km = isa ? AT : BT;
      const int W = isa ? BM : BN;
      const uint16_t* src;
      if (!km) {   // [row][64 k], 8 rows per piece
        const int row = 8 * fl + (lane >> 3);
        const int c = (lane & 7) ^ kc_swz(row);
        int64_t gr = r0 + row;
        gr = gr < R ? gr : R - 1;
        if constexpr (F8) {
          src = reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(X) + gr * ld + k0 + 16 * c);
        } else {
          // a chunk past K (K % 64 != 0, K % 8 == 0) reads the row's first chunk instead; the tail step zeroes it
          const int64_t kk = k0 + 8 * c < K ? k0 + 8 * c : 0;
          src = X + gr * ld + kk;
        }
      } else {     // [64 k][W cols], 1024 / (2 W) rows per piece
        const int byte = 1024 * fl + 16 * lane;
        const int row = byte / (2 * W);
        const int v = (byte % (2 * W)) >> 4;
        const int c = v ^ (km_swz8(row) >> 1);
        int64_t gk = k0 + row;
        gk = gk < K ? gk : K - 1;
        int64_t gc = r0 + 8 * c;
        gc = gc + 8 <= R ? gc : R - 8;
        src = X + gk * ld + gc;
      }
      uint16_t* dst = buf + (isa ? 0 : AIMG) + 512 * fl;
      __builtin_amdgcn_global_load_lds((bg_gl_void*)src, (bg_lds_void*)dst, 16, 0, 0);
    }
    if constexpr (F8) {   // waves 0 / 1: this stage's A / B scale bytes, 4 rows (16 B) per lane
      if (wave < 2) {
        const bool isa = wave == 0;
        const int64_t R = isa ? M : N, r0 = isa ? m0 : n0;
        int64_t r = r0 + 4 * lane;
        r = r + 4 <= R ? r : R - 4;
        const uint8_t* src = (isa ? p.xsa : p.xsb) + ((k0 / 128) * R + r) * 4;
        uint16_t* dst = buf + AIMG + BIMG + (isa ? 0 : 512);
        __builtin_amdgcn_global_load_lds((bg_gl_void*)src, (bg_lds_void*)dst, 16, 0, 0);
      }
    }
  };

  constexpr bool BIAS = EMODE == BG_ACCB;
  f32x4 acc[FM][FN];
  f32x4 accb[BIAS ? FM : 1];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if constexpr (BIAS) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool do_bias = BIAS && wc == 0 && tnn == 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;   // bf16(1.0)

  if (nk > 0) issue(0, 0);
  for (int t = 0; t < nk; ++t) {
    __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));   // vmcnt(0): this wave's pieces of step t landed
    __builtin_amdgcn_s_barrier();                              // ... every wave's; step t - 1's reads are done
    const int s = t & 1;
    const uint16_t* abuf = bg_lds + s * STAGE;
    const uint16_t* bbuf = abuf + AIMG;
    if constexpr (!F8) {
      const int64_t vr = K - kb - (int64_t)t * BG_BK;
      if (vr < BG_BK) {   // tail step
        if constexpr (AT || BT) {   // zero the k-major A (or B) rows past K (their DMA read clamped rows)
          uint16_t* z = bg_lds + s * STAGE + (AT ? 0 : AIMG);
          constexpr int ZW = AT ? BM : BN;
          for (int e = threadIdx.x; e < (BG_BK - (int)vr) * ZW; e += NW * 64) z[(int)vr * ZW + e] = 0;
        }
        if constexpr (!AT || !BT) {   // zero the k-contiguous images' 16-byte chunks past K (a row's first chunk)
          constexpr int ZR = (AT ? 0 : BM) + (BT ? 0 : BN);
          for (int e = threadIdx.x; e < ZR * 8; e += NW * 64) {
            const int row = e >> 3, pch = e & 7;
            const int c = pch ^ kc_swz(row < (AT ? 0 : BM) ? row : row - (AT ? 0 : BM));
            if (8 * c >= vr) {
              uint16_t* img = bg_lds + s * STAGE + (row < (AT ? 0 : BM) ? 0 : AIMG);
              const int rr = row < (AT ? 0 : BM) ? row : row - (AT ? 0 : BM);
              *reinterpret_cast<uint4*>(img + rr * BG_BK + 8 * pch) = make_uint4(0u, 0u, 0u, 0u);
            }
          }
        }
        __syncthreads();
      }
    }
    if (t + 1 < nk) issue(t + 1, s ^ 1);
    if constexpr (F8) {   // one block-scaled fp8 MFMA per accumulator tile covers the stage's 128 k
      bg_v8i af[FM], bfr[FN];
      int sca[FM], scb[FN];
      // lane l supplies the scale byte of row l & 15, block l >> 4 (frag_kc8's map)
      const uint8_t* sbuf = reinterpret_cast<const uint8_t*>(abuf + AIMG + BIMG);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        af[i] = frag_kc8(abuf, wr * WTM + 16 * i, lane);
        const uint32_t sa_ = lds_addr(sbuf + (wr * WTM + 16 * i + (lane & 15)) * 4 + (lane >> 4));
        asm volatile("ds_read_u8 %0, %1" : "=v"(sca[i]) : "v"(sa_));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        bfr[j] = frag_kc8(bbuf, wc * WTN + 16 * j, lane);
        const uint32_t sb_ = lds_addr(sbuf + 1024 + (wc * WTN + 16 * j + (lane & 15)) * 4 + (lane >> 4));
        asm volatile("ds_read_u8 %0, %1" : "=v"(scb[j]) : "v"(sb_));
      }
      lgkm_wait<0>();
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" : "+v"(af[i]), "+v"(sca[i]));
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" : "+v"(bfr[j]), "+v"(scb[j]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, sca[i], 0,
                                                                       scb[j]);
      continue;
    }
    // fragment reads of a k half, then its MFMAs; with registers to spare (<= 16 accumulator tiles per wave) the
    // second half's reads are issued before the first half's MFMAs, so their LDS latency hides behind them
    auto read_frags = [&](int hh, bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wr * WTM + 16 * i;
        if constexpr (AT) af[i] = frag_km<BM>(abuf, r, hh, lane);
        else af[i] = frag_kc(abuf, r, hh, lane);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wc * WTN + 16 * j;
        if constexpr (BT) bfr[j] = frag_km<BN>(bbuf, c, hh, lane);
        else bfr[j] = frag_kc(bbuf, c, hh, lane);
      }
    };
    auto tie = [&](bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" : "+v"(bfr[j]));
      __builtin_amdgcn_sched_barrier(0);
    };
    auto mfmas = [&](bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if constexpr (BIAS)
          if (do_bias) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, accb[i], 0, 0, 0);
      }
    };
    constexpr bool PIPE = FM * FN <= 16;
    if constexpr (PIPE) {
      bf16x8 a0[FM], b0[FN], a1[FM], b1[FN];
      read_frags(0, a0, b0);
      lgkm_wait<0>();
      read_frags(1, a1, b1);
      tie(a0, b0);
      mfmas(a0, b0);
      lgkm_wait<0>();
      tie(a1, b1);
      mfmas(a1, b1);
    } else {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        bf16x8 af[FM], bfr[FN];
        read_frags(hh, af, bfr);
        lgkm_wait<0>();
        tie(af, bfr);
        mfmas(af, bfr);
      }
    }
  }

  // ---- epilogue ----
  const GemmP& g = p.g;
  float alpha = g.alpha;

  if constexpr (EMODE == BG_ACC || EMODE == BG_ACCB) {
    if (p.splits > 1) {   // raw partials of this split (plain stores; big_fold_kernel adds them in split order)
      float* w = p.ws + (int64_t)sp * M * N;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int64_t mb = m0 + wr * WTM + 16 * i + 4 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int64_t n = n0 + wc * WTN + 16 * j + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (mb + r < M && n < N) w[(mb + r) * N + n] = acc[i][j][r];
        }
        if constexpr (BIAS) {
          if (do_bias && (lane & 15) == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (mb + r < M) p.wsb[(int64_t)sp * M + mb + r] = accb[i][r];
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int64_t mb = m0 + wr * WTM + 16 * i + 4 * (lane >> 4);
      float old[FN][4];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = n0 + wc * WTN + 16 * j + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) old[j][r] = (mb + r < M && n < N) ? g.C[(mb + r) * g.sCm + n * g.sCn] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = n0 + wc * WTN + 16 * j + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (mb + r < M && n < N) g.C[(mb + r) * g.sCm + n * g.sCn] = old[j][r] + alpha * acc[i][j][r];
      }
      if constexpr (BIAS) {
        if (do_bias && (lane & 15) == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (mb + r < M) p.ones_out[mb + r] += alpha * accb[i][r];
        }
      }
    }
    return;
  } else {
  const int epi = g.epi;
  const uint64_t seed = (epi & KDFM_EPI_DROPOUT) ? load_seed(g.seed) : 0ull;
  const float keep_scale = (epi & KDFM_EPI_DROPOUT) ? 1.f / (1.f - g.dropout_p) : 1.f;
  bool single;
  const float* side = epi_side_src(g, single);
  float mse_part = 0.f;
  auto epi1 = [&](int64_t m, int64_t n, float a, float bnv, float svv, bool rokv, float& pre) -> float {
    if constexpr (EMODE == BG_DSILU_DROP) {
      float v = a;
      if (epi & KDFM_EPI_DROPOUT) {
        const uint64_t idx = (uint64_t)m * (uint64_t)N + (uint64_t)n;
        v = dropout_keep(seed, g.rng_stream, idx, g.dropout_p) ? v * keep_scale : 0.f;
      }
      return v * dsiluf_(svv);
    } else {
      return skc_epi<EMODE>(g, m, n, a, bnv, svv, rokv, seed, keep_scale, mse_part, pre, 0);
    }
  };
  // Row-contiguous epilogue: each 16-row strip of the wave's tile is transposed through LDS (free after the main
  // loop) so a lane finishes 4 consecutive columns of one row -- 16-byte side-operand loads and output stores,
  // 16 lanes per 256-byte row segment (the accumulator layout gives a lane 4 rows of one column: 4-byte stores).
  constexpr int SLD = WTN + 4;   // strip row stride (floats)
  const uintptr_t al = (uintptr_t)(p.C16 ? (const void*)p.C16 : (const void*)g.C) |
                       (uintptr_t)((epi & KDFM_EPI_STORE_PRE) ? g.Cpre : nullptr) | (uintptr_t)side |
                       (uintptr_t)((epi & KDFM_EPI_BIAS) ? g.bias : nullptr);
  const bool vec = (N % 4) == 0 && g.sCn == 1 && (g.sCm % 4) == 0 && (al & (p.C16 ? 7 : 15)) == 0 &&
                   (((uintptr_t)g.Cpre | (uintptr_t)side | (uintptr_t)g.bias) & 15) == 0;
  if (vec) {
    __syncthreads();   // every wave has finished reading the last stage: the LDS is reused below
    float* strip = reinterpret_cast<float*>(bg_lds) + wave * (16 * SLD);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) strip[(4 * (lane >> 4) + r) * SLD + 16 * j + (lane & 15)] = acc[i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      constexpr int C4 = WTN / 4;   // float4 groups per strip row
#pragma unroll
      for (int q = 0; q < 16 * C4 / 64; ++q) {
        const int f = q * 64 + lane;
        const int row = f / C4, c4 = f % C4;
        const float4 a4 = *reinterpret_cast<const float4*>(strip + row * SLD + 4 * c4);
        const int64_t m = m0 + wr * WTM + 16 * i + row;
        const int64_t n = n0 + wc * WTN + 4 * c4;
        if (m >= M || n >= N) continue;
        const int64_t off = m * g.sCm + n;
        float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f), s4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (epi & KDFM_EPI_BIAS) b4 = *reinterpret_cast<const float4*>(g.bias + n);
        if (side) s4 = *reinterpret_cast<const float4*>(side + off);
        const bool rokv = epi_row_ok(g, m);
        float pre[4] = {0.f, 0.f, 0.f, 0.f};
        const float o0 = epi1(m, n + 0, alpha * a4.x, b4.x, s4.x, rokv, pre[0]);
        const float o1 = epi1(m, n + 1, alpha * a4.y, b4.y, s4.y, rokv, pre[1]);
        const float o2 = epi1(m, n + 2, alpha * a4.z, b4.z, s4.z, rokv, pre[2]);
        const float o3 = epi1(m, n + 3, alpha * a4.w, b4.w, s4.w, rokv, pre[3]);
        if (epi & KDFM_EPI_STORE_PRE) *reinterpret_cast<float4*>(g.Cpre + off) = make_float4(pre[0], pre[1], pre[2], pre[3]);
        if (p.C16) {
          uint2 h;
          h.x = pack_bf16x2(o0, o1);
          h.y = pack_bf16x2(o2, o3);
          *reinterpret_cast<uint2*>(p.C16 + off) = h;
        } else {
          *reinterpret_cast<float4*>(g.C + off) = make_float4(o0, o1, o2, o3);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this strip's reads are done before the next writes
    }
    return;
  }
  float bn[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t n = n0 + wc * WTN + 16 * j + (lane & 15);
    bn[j] = ((epi & KDFM_EPI_BIAS) && n < N) ? g.bias[n] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int64_t mb = m0 + wr * WTM + 16 * i + 4 * (lane >> 4);
    bool rok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rok[r] = mb + r < M && epi_row_ok(g, mb + r < M ? mb + r : 0);
    // side operands a column tile at a time when the epilogue is the generic one (its flag walk holds more
    // registers beside the 4 * FM * FN accumulators), else all of the row tile's first
    constexpr int SVJ = EMODE == SKC_EPI_GENERIC ? 1 : FN;
#pragma unroll
    for (int j0 = 0; j0 < FN; j0 += SVJ) {
    float sv[SVJ][4];
#pragma unroll
    for (int jj = 0; jj < SVJ; ++jj) {
      const int64_t n = n0 + wc * WTN + 16 * (j0 + jj) + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[jj][r] = (side && mb + r < M && n < N) ? side[(mb + r) * g.sCm + n * g.sCn] : 0.f;
    }
#pragma unroll
    for (int jj = 0; jj < SVJ; ++jj) {
      const int j = j0 + jj;
      const int64_t n = n0 + wc * WTN + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = mb + r;
        if (m >= M || n >= N) continue;
        const int64_t off = m * g.sCm + n * g.sCn;
        float pre = 0.f;
        const float v = epi1(m, n, alpha * acc[i][j][r], bn[j], sv[jj][r], rok[r], pre);
        if (epi & KDFM_EPI_STORE_PRE) g.Cpre[off] = pre;
        if (p.C16) p.C16[off] = f2bf(v);
        else g.C[off] = v;
      }
    }
    }
  }
  }
}

// C[m][n] += alpha sum_s ws[s][m][n] (s in order), 4 columns per thread; then ones_out[m] += alpha sum_s wsb[s][m]
__global__ __launch_bounds__(256) void big_fold_kernel(float* C, int64_t sCm, const float* ws, const float* wsb,
                                                       float* ones, int64_t M, int64_t N, int S, float alpha) {
  const int64_t n4 = N / 4, MN = M * N;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < M * n4) {
    const int64_t m = e / n4, n = (e - m * n4) * 4;
    float4 a = *reinterpret_cast<const float4*>(ws + m * N + n);
    for (int s = 1; s < S; ++s) {
      const float4 b = *reinterpret_cast<const float4*>(ws + s * MN + m * N + n);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float* c = C + m * sCm + n;
    c[0] += alpha * a.x; c[1] += alpha * a.y; c[2] += alpha * a.z; c[3] += alpha * a.w;
  } else if (ones && e - M * n4 < M) {
    const int64_t m = e - M * n4;
    float a = wsb[m];
    for (int s = 1; s < S; ++s) a += wsb[s * M + m];
    ones[m] += alpha * a;
  }
}

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EMODE, bool F8 = false>
int big_launch(const BigP& p, hipStream_t st) {
  auto kern = big_gemm_kernel<BM, BN, WM, WN, AT, BT, EMODE, F8>;
  constexpr int lds = 2 * ((BM + BN) * BG_BK + (F8 ? 1024 : 0)) * 2;   // two stages (big_gemm_kernel's STAGE)
  static const bool once = [&] {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return true;
  }();
  (void)once;
  const int64_t tm = ceil_div(p.g.M, BM), tn = ceil_div(p.g.N, BN);
  BigP q = p;
  q.tn = (int)tn;
  if (q.splits < 1) q.splits = 1;
  q.kchunk = ceil_div(ceil_div(p.g.K, q.splits), BG_BK) * BG_BK;
  if (F8) q.kchunk = p.g.K;
  hipLaunchKernelGGL(kern, dim3((unsigned)(tm * tn * q.splits)), dim3(WM * WN * 64), lds, st, q);
  int rc = check_launch("kdfm_gemm_big");
  if (rc || q.splits == 1) return rc;
  const int64_t n = p.g.M * (p.g.N / 4) + (p.ones_out ? p.g.M : 0);
  hipLaunchKernelGGL(big_fold_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, p.g.C, p.g.sCm, q.ws, q.wsb,
                     p.ones_out, p.g.M, p.g.N, q.splits, p.g.alpha);
  return check_launch("kdfm_gemm_big (split fold)");
}

// compile-time epilogue per layout (the generic instance covers every flag set)
template <int BM, int BN, int WM, int WN, bool AT, bool BT>
int big_epi(const BigP& p, hipStream_t st) {
  if constexpr (AT && BT) {   // the weight-gradient layout: accumulate only
    if constexpr (BM == 256 && BN == 256) {   // big_dispatch never asks it for the bias gradient (spills)
      return p.ones_out ? KDFM_EUNSUPPORTED : big_launch<BM, BN, WM, WN, AT, BT, BG_ACC>(p, st);
    } else {
      return p.ones_out ? big_launch<BM, BN, WM, WN, AT, BT, BG_ACCB>(p, st)
                        : big_launch<BM, BN, WM, WN, AT, BT, BG_ACC>(p, st);
    }
  } else {
  if ((p.g.epi & ~KDFM_EPI_DROPOUT) == KDFM_EPI_DSILU) return big_launch<BM, BN, WM, WN, AT, BT, BG_DSILU_DROP>(p, st);
  const int em = skc_epi_mode(p.g.epi);
  switch (em) {
    case SKC_EPI_NONE: return big_launch<BM, BN, WM, WN, AT, BT, SKC_EPI_NONE>(p, st);
    case SKC_EPI_SILU_DROP: return big_launch<BM, BN, WM, WN, AT, BT, SKC_EPI_SILU_DROP>(p, st);
    case SKC_EPI_DROP_RESID: return big_launch<BM, BN, WM, WN, AT, BT, SKC_EPI_DROP_RESID>(p, st);
    case SKC_EPI_RESID: return big_launch<BM, BN, WM, WN, AT, BT, SKC_EPI_RESID>(p, st);
    default:
      if constexpr (BM == 256 && BN == 256) return KDFM_EUNSUPPORTED;   // big_dispatch never picks it (spills)
      else return big_launch<BM, BN, WM, WN, AT, BT, SKC_EPI_GENERIC>(p, st);
  }
  }
}

// fp8 instances: the forward and data-gradient products (k-contiguous operands), 256 x 128 / 128 x 128 tiles
template <int BM, int BN, int WM, int WN>
int big_epi_f8(const BigP& p, hipStream_t st) {
  if ((p.g.epi & ~KDFM_EPI_DROPOUT) == KDFM_EPI_DSILU)
    return big_launch<BM, BN, WM, WN, false, false, BG_DSILU_DROP, true>(p, st);
  switch (skc_epi_mode(p.g.epi)) {
    case SKC_EPI_NONE: return big_launch<BM, BN, WM, WN, false, false, SKC_EPI_NONE, true>(p, st);
    case SKC_EPI_SILU_DROP: return big_launch<BM, BN, WM, WN, false, false, SKC_EPI_SILU_DROP, true>(p, st);
    case SKC_EPI_DROP_RESID: return big_launch<BM, BN, WM, WN, false, false, SKC_EPI_DROP_RESID, true>(p, st);
    case SKC_EPI_RESID: return big_launch<BM, BN, WM, WN, false, false, SKC_EPI_RESID, true>(p, st);
    default: return big_launch<BM, BN, WM, WN, false, false, SKC_EPI_GENERIC, true>(p, st);
  }
}

// does the compile-time epilogue set cover this descriptor (else the generic instance, which the 256 x 256 tile
// does not carry: its flag walk beside 128 accumulators spills)
bool big_epi_compiled(const BigP& p) {
  if (p.accum) return true;
  if ((p.g.epi & ~KDFM_EPI_DROPOUT) == KDFM_EPI_DSILU) return true;
  const int em = skc_epi_mode(p.g.epi);
  return em == SKC_EPI_NONE || em == SKC_EPI_SILU_DROP || em == SKC_EPI_DROP_RESID || em == SKC_EPI_RESID;
}

// tile shape: the one whose whole-chip rounds (tiles / 256 CUs, rounded up) times its per-tile MFMA work is least
// (a 256x256 tile does 4x a 128x128 one's work at about 1.15x its rate per CU; 256x128 in between)
int big_pick(int64_t M, int64_t N) {
  const double eff[3] = {1.0, 0.93, 0.85};   // relative per-CU rate: 256x256, 256x128, 128x128
  const int bm[3] = {256, 256, 128}, bn[3] = {256, 128, 128};
  int best = 0;
  double bt = 1e300;
  for (int c = 0; c < 3; ++c) {
    const int64_t tiles = ceil_div(M, bm[c]) * ceil_div(N, bn[c]);
    const double rounds = (double)ceil_div(tiles, 256);
    const double t = rounds * (double)bm[c] * bn[c] / eff[c];
    if (t < bt - 1e-9) {
      bt = t;
      best = c;
    }
  }
  return best;
}

// weight-gradient layout: the 256 x 128 tile, and split reductions when its tiles alone leave CUs idle (at least 8
// K steps per split, at most 8 splits); KDFM_BIG_SPLIT forces a count
int big_splits(int64_t M, int64_t N, int64_t K) {
  const char* e = getenv("KDFM_BIG_SPLIT");
  const int64_t tiles = ceil_div(M, 256) * ceil_div(N, 128);
  int64_t S = e ? atoi(e) : (256 + tiles / 2) / tiles;
  const int64_t smax = K / (8 * BG_BK);
  if (S > 8) S = 8;
  if (S > smax) S = smax;
  if ((N % 4) != 0) S = 1;
  return S < 1 ? 1 : (int)S;
}

template <bool AT, bool BT>
int big_dispatch(BigP p, hipStream_t st) {
  const char* e = getenv("KDFM_BIG_TILE");   // 0 / 1 / 2 forces a tile shape (A/B probes)
  int c = e ? atoi(e) : big_pick(p.g.M, p.g.N);
  if (AT && BT) {
    if (!e) c = 1;
    const int S = big_splits(p.g.M, p.g.N, p.g.K);
    const int64_t need = (int64_t)S * p.g.M * p.g.N + (int64_t)S * p.g.M;
    if (S > 1 && p.g.ws && p.g.ws_len >= need && p.g.sCn == 1) {
      p.splits = S;
      p.ws = p.g.ws;
      p.wsb = p.g.ws + (int64_t)S * p.g.M * p.g.N;
    }
  }
  // the 256 x 256 tile has no generic-epilogue instance, and its bias-gradient accumulators spill
  if (c == 0 && (!big_epi_compiled(p) || p.ones_out)) c = 1;
  if (c == 0) return big_epi<256, 256, 2, 4, AT, BT>(p, st);
  if (c == 1) return big_epi<256, 128, 4, 2, AT, BT>(p, st);
  return big_epi<128, 128, 2, 2, AT, BT>(p, st);
}

__device__ __forceinline__ float bg_load(const void* src, int bf, int64_t i) {
  return bf ? __uint_as_float(((uint32_t) reinterpret_cast<const uint16_t*>(src)[i]) << 16)
            : reinterpret_cast<const float*>(src)[i];
}

// ---- MX fp8 quantisation (OCP e4m3, e8m0 block scales over 32 consecutive k) ----
// block exponent e = ceil(log2(amax / 448)) (clamped to the e8m0 range): every element of the block is then
// exactly x 2^-e <= 448 in magnitude, no saturation; q = e4m3(x 2^-e) (round to nearest even), scale byte e + 127
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  int ex;
  const float m = frexpf(amax * (1.f / 448.f), &ex);   // amax / 448 = m 2^ex, m in [0.5, 1)
  int e = m > 0.5f ? ex : ex - 1;
  if (ldexpf(amax, -e) > 448.f) ++e;   // the 1/448 product's rounding
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}
__device__ __forceinline__ uint32_t mx_q4(float a, float b, float c, float d, int e) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(a, -e), ldexpf(b, -e), 0, false) & 0xFFFFu;
  const uint32_t hi = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(c, -e), ldexpf(d, -e), 0, false) & 0xFFFFu;
  return lo | (hi << 16);
}

// row-major: block (row, kb) = src[row][32 kb .. +31]; 8 lanes per block, 4 elements each
__global__ __launch_bounds__(256) void mx_quant_kernel(const void* src, int bf, int64_t rows, int64_t cols, int64_t ld,
                                                       uint8_t* dst, int64_t ldd, uint8_t* xs) {
  const int64_t nkb = cols / 32, nblk = rows * nkb;
  const int sub = threadIdx.x & 7;
  for (int64_t blk = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3; blk < nblk + 0; blk += (int64_t)gridDim.x * 32) {
    const int64_t r = blk / nkb, kb = blk - r * nkb;
    const int64_t o = r * ld + 32 * kb + 4 * sub;
    float v[4];
    if (bf) {
      const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(src) + o);
      v[0] = __uint_as_float(w.x << 16); v[1] = __uint_as_float(w.x & 0xFFFF0000u);
      v[2] = __uint_as_float(w.y << 16); v[3] = __uint_as_float(w.y & 0xFFFF0000u);
    } else {
      const float4 w = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src) + o);
      v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
    }
    float m = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    m = fmaxf(m, __shfl_xor(m, 1, 64));
    m = fmaxf(m, __shfl_xor(m, 2, 64));
    m = fmaxf(m, __shfl_xor(m, 4, 64));
    const int e = mx_exp(m);
    *reinterpret_cast<uint32_t*>(dst + r * ldd + 32 * kb + 4 * sub) = mx_q4(v[0], v[1], v[2], v[3], e);
    if (sub == 0) xs[((kb >> 2) * rows + r) * 4 + (kb & 3)] = (uint8_t)(e + 127);
  }
}

// row-major, 16-byte rows (ld a multiple of 8 bf16 / 4 f32 elements, 16-byte aligned base): a workgroup pass is
// 16 rows x one 128-column stage; a thread owns 8 consecutive elements (one 16-byte load of bf16, two of f32), 4
// threads one MX block, 16 one stage row: each row's 128 output bytes and the 16 rows' 64 scale bytes (contiguous
// in the stage-major layout) are written whole by the pass -- the 8-lanes-per-block kernel above wrote them in
// 4-byte pieces and single scale bytes scattered over the stages
__device__ __forceinline__ void mxr_load(const void* src, int bf, int64_t o, float (&v)[8]) {
  if (bf) {
    const uint4 w = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(src) + o);
    const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src) + o);
    const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src) + o + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

// MXR_U tiles per loop iteration (their loads issued together), over a grid of at most a few workgroups per CU:
// one tile per workgroup made the launch dispatch-bound (12 864 workgroups of 4 KB each at 6432 x 4096)
constexpr int MXR_U = 4;

__global__ __launch_bounds__(256) void mx_quant_rows_kernel(const void* src, int bf, int64_t rows, int64_t cols,
                                                            int64_t ld, uint8_t* dst, int64_t ldd, uint8_t* xs) {
  const int64_t nrt = (rows + 15) / 16, nt = nrt * (cols / 128);
  const int j = threadIdx.x & 15;
  for (int64_t t0 = blockIdx.x; t0 < nt; t0 += (int64_t)MXR_U * gridDim.x) {
    float v[MXR_U][8];
    int64_t s[MXR_U], r[MXR_U];
    bool ok[MXR_U];
#pragma unroll
    for (int u = 0; u < MXR_U; ++u) {
      const int64_t t = t0 + (int64_t)u * gridDim.x;
      const int64_t tt = t < nt ? t : 0;
      s[u] = tt / nrt;
      r[u] = (tt - s[u] * nrt) * 16 + (threadIdx.x >> 4);
      ok[u] = t < nt && r[u] < rows;
      mxr_load(src, bf, (ok[u] ? r[u] : 0) * ld + 128 * s[u] + 8 * j, v[u]);
    }
#pragma unroll
    for (int u = 0; u < MXR_U; ++u) {
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) m = fmaxf(m, fabsf(v[u][i]));
      m = fmaxf(m, __shfl_xor(m, 1, 64));
      m = fmaxf(m, __shfl_xor(m, 2, 64));
      const int e = mx_exp(m);
      if (ok[u]) {
        uint2 w;
        w.x = mx_q4(v[u][0], v[u][1], v[u][2], v[u][3], e);
        w.y = mx_q4(v[u][4], v[u][5], v[u][6], v[u][7], e);
        *reinterpret_cast<uint2*>(dst + r[u] * ldd + 128 * s[u] + 8 * j) = w;
        if ((j & 3) == 0) xs[(s[u] * rows + r[u]) * 4 + (j >> 2)] = (uint8_t)(e + 127);
      }
    }
  }
}

// transposed (the data gradient's W^T rows): output row c = source column c, blocks over 32 source rows; a 32 x 64
// source tile through LDS, 4 lanes per output block (8 elements each)
__global__ __launch_bounds__(256) void mx_quant_t_kernel(const void* src, int bf, int64_t rows, int64_t cols,
                                                         int64_t ld, uint8_t* dst, int64_t ldd, uint8_t* xs) {
  __shared__ float tile[32][65];
  const int64_t tr = rows / 32, tc = ceil_div(cols, 64);
  for (int64_t t = blockIdx.x; t < tr * tc; t += gridDim.x) {
    const int64_t r0 = (t / tc) * 32, c0 = (t % tc) * 64;
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int rr = e / 64, cc = e % 64;
      tile[rr][cc] = c0 + cc < cols ? bg_load(src, bf, (r0 + rr) * ld + c0 + cc) : 0.f;
    }
    __syncthreads();
    const int cc = threadIdx.x >> 2, q = threadIdx.x & 3;   // output row c0 + cc, elements 8 q .. + 7 of the block
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tile[8 * q + i][cc];
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) m = fmaxf(m, fabsf(v[i]));
    m = fmaxf(m, __shfl_xor(m, 1, 64));
    m = fmaxf(m, __shfl_xor(m, 2, 64));
    const int e = mx_exp(m);
    if (c0 + cc < cols) {
      uint2 w;
      w.x = mx_q4(v[0], v[1], v[2], v[3], e);
      w.y = mx_q4(v[4], v[5], v[6], v[7], e);
      *reinterpret_cast<uint2*>(dst + (c0 + cc) * ldd + r0 + 8 * q) = w;
      const int64_t kb = r0 / 32;
      if (q == 0) xs[((kb >> 2) * cols + c0 + cc) * 4 + (kb & 3)] = (uint8_t)(e + 127);
    }
    __syncthreads();
  }
}

__global__ void cast2d_kernel(const float* __restrict__ src, int64_t lds, uint16_t* __restrict__ dst, int64_t ldd,
                              int64_t rows, int64_t cols) {
  const int64_t c4 = cols / 4;
  const int64_t n = rows * c4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / c4, c = (i - r * c4) * 4;
    const float4 v = *reinterpret_cast<const float4*>(src + r * lds + c);
    uint2 o;
    o.x = pack_bf16x2(v.x, v.y);
    o.y = pack_bf16x2(v.z, v.w);
    *reinterpret_cast<uint2*>(dst + r * ldd + c) = o;
  }
}

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_gemm_big_ws(int64_t M, int64_t N, int64_t K, int layout) {
  using namespace kdfm;
  if (layout != KDFM_BIG_TN || !kdfm_gemm_big_supported(M, N, K, layout)) return 0;
  const int S = big_splits(M, N, K);
  return S > 1 ? (int64_t)S * M * N + (int64_t)S * M : 0;
}

int kdfm_gemm_big_supported(int64_t M, int64_t N, int64_t K, int layout) {
  using namespace kdfm;
  if (M < 64 || N < 64 || K < 64 || layout < 0 || layout > 2) return 0;
  if (layout == KDFM_BIG_NT || layout == KDFM_BIG_NN) {
    if (K % 8) return 0;   // the k-contiguous images' tail step zeroes whole 16-byte chunks
  }
  if (layout == KDFM_BIG_NN && N % 8) return 0;
  if (layout == KDFM_BIG_TN && (M % 8 || N % 8)) return 0;
  return 1;
}

int kdfm_gemm_big(const kdfm_gemm_desc* d, const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int layout,
                  uint16_t* C16, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(d && A && B, "null argument");
  KDFM_REQUIRE(kdfm_gemm_big_supported(d->M, d->N, d->K, layout), "shape / layout not supported by the big-tile GEMM");
  KDFM_REQUIRE(d->batch1 == 1 && d->batch2 == 1 && d->splitk == 1, "unbatched, no split-K");
  KDFM_REQUIRE(((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0 && lda % 8 == 0 && ldb % 8 == 0,
               "operands 16-byte aligned with row strides multiple of 8 elements");
  const bool accum = d->epi == KDFM_EPI_ATOMIC;
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_MSE), "the MSE epilogue is not supported here");
  KDFM_REQUIRE(accum ? (C16 == nullptr && d->C != nullptr) : (d->C != nullptr || C16 != nullptr),
               "accumulate mode needs the f32 C; otherwise C or C16");
  KDFM_REQUIRE(d->ones_out == nullptr || accum, "the bias-gradient output needs accumulate mode");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_BIAS) || d->bias, "EPI_BIAS without bias");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_RESID) || d->R, "EPI_RESID without R");
  KDFM_REQUIRE(!(d->epi & (KDFM_EPI_DRELU | KDFM_EPI_DSILU)) || d->aux, "derivative epilogue without aux");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_STORE_PRE) || d->Cpre, "EPI_STORE_PRE without Cpre");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_BETA) || (d->C && !C16), "EPI_BETA reads the f32 C");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_ROWMASK) || (d->mask_len && d->mask_T > 0 && d->mask_div > 0), "ROWMASK fields");
  BigP p{};
  p.A = A; p.B = B; p.lda = lda; p.ldb = ldb; p.C16 = C16;
  p.accum = accum ? 1 : 0;
  p.ones_out = d->ones_out;
  GemmP& g = p.g;
  g.C = d->C; g.bias = d->bias; g.R = d->R; g.aux = d->aux; g.Cpre = d->Cpre;
  g.M = d->M; g.N = d->N; g.K = d->K;
  g.sCm = d->sCm; g.sCn = d->sCn;
  g.alpha = d->alpha; g.beta = d->beta; g.rscale = d->rscale; g.dropout_p = d->dropout_p;
  g.seed = d->seed; g.rng_stream = d->rng_stream;
  g.epi = accum ? 0 : d->epi;
  g.mask_len = d->mask_len; g.mask_T = d->mask_T; g.mask_div = d->mask_div;
  g.ones_col = -1;
  g.ws = d->ws; g.ws_len = d->ws_len;
  p.splits = 1;
  bool single;
  (void)epi_side_src(g, single);
  KDFM_REQUIRE(single, "at most one side operand (R, aux or C) per epilogue");
  hipStream_t st = as_stream(stream);
  set_route(ROUTE_BIG);
  if (d->M == 0 || d->N == 0) return KDFM_OK;
  KDFM_REQUIRE(accum == (layout == KDFM_BIG_TN), "the TN (weight-gradient) layout accumulates; NT / NN do not");
  switch (layout) {
    case KDFM_BIG_NT: return big_dispatch<false, false>(p, st);
    case KDFM_BIG_NN: return big_dispatch<false, true>(p, st);
    default: return big_dispatch<true, true>(p, st);
  }
}

int kdfm_fp8_quant_mx(const void* src, int src_bf16, int64_t rows, int64_t cols, int64_t ld, uint8_t* dst, int64_t ldd,
                      uint8_t* scales, int transpose, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(src && dst && scales && rows > 0 && cols > 0 && ld >= cols, "bad arguments");
  const int64_t kdim = transpose ? rows : cols;   // the contraction length the 32-blocks run along
  KDFM_REQUIRE(kdim % 128 == 0 && ld % 4 == 0 && ldd % 16 == 0, "contraction length % 128, ld % 4, ldd % 16");
  KDFM_REQUIRE(transpose ? ldd >= rows : (ldd >= cols && (((uintptr_t)src) & (src_bf16 ? 7 : 15)) == 0),
               "layout / alignment");
  hipStream_t st = as_stream(stream);
  if (transpose) {
    const int64_t tiles = (rows / 32) * ceil_div(cols, 64);
    hipLaunchKernelGGL(mx_quant_t_kernel, dim3((unsigned)(tiles < 8192 ? tiles : 8192)), dim3(256), 0, st, src,
                       src_bf16, rows, cols, ld, dst, ldd, scales);
  } else if (((((uintptr_t)src) & 15) == 0) && ld % (src_bf16 ? 8 : 4) == 0) {
    const int64_t tiles = ceil_div(rows, 16) * (cols / 128);
    static const int64_t cap = [] { const char* e = getenv("KDFM_MXQ_GRID"); return e ? atoll(e) : 2048LL; }();
    const int64_t g = ceil_div(tiles, MXR_U);
    hipLaunchKernelGGL(mx_quant_rows_kernel, dim3((unsigned)(g < cap ? g : cap)), dim3(256), 0, st, src,
                       src_bf16, rows, cols, ld, dst, ldd, scales);
  } else {
    const int64_t blocks = ceil_div(rows * (cols / 32), 32);
    hipLaunchKernelGGL(mx_quant_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, st, src,
                       src_bf16, rows, cols, ld, dst, ldd, scales);
  }
  return check_launch("kdfm_fp8_quant_mx");
}

int kdfm_gemm_big_fp8(const kdfm_gemm_desc* d, const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb,
                      const uint8_t* sa, const uint8_t* sb, uint16_t* C16, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(d && A && B, "null argument");
  KDFM_REQUIRE(d->M >= 128 && d->N >= 128 && d->K >= 128 && d->K % 128 == 0 && d->M % 4 == 0 && d->N % 4 == 0,
               "fp8 route: M, N >= 128 (multiples of 4), K % 128 == 0");
  KDFM_REQUIRE(sa && sb, "the MX scale tensors are required");
  KDFM_REQUIRE(d->batch1 == 1 && d->batch2 == 1 && d->splitk == 1 && d->epi != KDFM_EPI_ATOMIC,
               "unbatched forward / data-gradient products only");
  KDFM_REQUIRE(((((uintptr_t)A) | ((uintptr_t)B)) & 15) == 0 && lda % 16 == 0 && ldb % 16 == 0,
               "operands 16-byte aligned, row strides multiples of 16 bytes");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_MSE) && (d->C != nullptr || C16 != nullptr), "C or C16; no MSE");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_BIAS) || d->bias, "EPI_BIAS without bias");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_RESID) || d->R, "EPI_RESID without R");
  KDFM_REQUIRE(!(d->epi & (KDFM_EPI_DRELU | KDFM_EPI_DSILU)) || d->aux, "derivative epilogue without aux");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_STORE_PRE) || d->Cpre, "EPI_STORE_PRE without Cpre");
  KDFM_REQUIRE(!(d->epi & KDFM_EPI_BETA) || (d->C && !C16), "EPI_BETA reads the f32 C");
  BigP p{};
  p.A = reinterpret_cast<const uint16_t*>(A);
  p.B = reinterpret_cast<const uint16_t*>(B);
  p.lda = lda; p.ldb = ldb; p.C16 = C16; p.xsa = sa; p.xsb = sb; p.splits = 1;
  GemmP& g = p.g;
  g.C = d->C; g.bias = d->bias; g.R = d->R; g.aux = d->aux; g.Cpre = d->Cpre;
  g.M = d->M; g.N = d->N; g.K = d->K;
  g.sCm = d->sCm; g.sCn = d->sCn;
  g.alpha = d->alpha; g.beta = d->beta; g.rscale = d->rscale; g.dropout_p = d->dropout_p;
  g.seed = d->seed; g.rng_stream = d->rng_stream; g.epi = d->epi;
  g.mask_len = d->mask_len; g.mask_T = d->mask_T; g.mask_div = d->mask_div;
  g.ones_col = -1;
  bool single;
  (void)epi_side_src(g, single);
  KDFM_REQUIRE(single, "at most one side operand (R, aux or C) per epilogue");
  set_route(ROUTE_BIG);
  hipStream_t st = as_stream(stream);
  const char* e = getenv("KDFM_BIG_TILE");
  int c = e ? atoi(e) : big_pick(d->M, d->N);
  if (c == 0) c = 1;   // the 256 x 256 fp8 tile's fragments do not fit beside its accumulators
  return c == 1 ? big_epi_f8<256, 128, 4, 2>(p, st) : big_epi_f8<128, 128, 2, 2>(p, st);
}

int kdfm_cast_bf16_2d(const float* src, int64_t lds, uint16_t* dst, int64_t ldd, int64_t rows, int64_t cols,
                      void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(src && dst && rows >= 0 && cols >= 0, "bad arguments");
  KDFM_REQUIRE(cols % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0 && (((uintptr_t)src) & 15) == 0 &&
                   (((uintptr_t)dst) & 7) == 0,
               "cols / strides multiples of 4, src 16-B / dst 8-B aligned");
  if (rows == 0 || cols == 0) return KDFM_OK;
  const int64_t n = rows * (cols / 4);
  const int64_t blocks = ceil_div(n, 256) < 8192 ? ceil_div(n, 256) : 8192;
  hipLaunchKernelGGL(cast2d_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), src, lds, dst, ldd, rows,
                     cols);
  return check_launch("kdfm_cast_bf16_2d");
}

}  // extern "C"
