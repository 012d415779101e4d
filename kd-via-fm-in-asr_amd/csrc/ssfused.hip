// Striding ConvSubsampling forward in ONE kernel (bf16 MFMA mode): conv1 computed on the fly into LDS,
// conv2 as an implicit GEMM over it.  The conv1 output y1 (4x the positions of the output, C channels:
// 361 MB bf16 for the teacher at B = 32, 16 s) never makes an HBM round trip.
//
// Reference: ConvSubsampling(subsampling='striding', factor 4, conv_channels = d), built
// conformer_encoder.py:381-390, called :635 (source absent):
//   x (B,T,80) -> Conv2d(1->C, 3x3, s2, p1) -> ReLU -> Conv2d(C->C, 3x3, s2, p1) -> ReLU,
// padded frames masked to zero before each conv (mel rows >= mel_len, y1 rows >= len1) and the output
// rows >= len2 zeroed (the A.3 mask flag, default on).
//
// One workgroup (8 waves) = one utterance x R output rows (t2) x all 20 frequency columns x all C output
// channels.  Per workgroup:
//   prologue: the mel patch it reads (4R+3 rows x 82 columns, zero outside the utterance / the frame
//     mask) is staged in LDS, then turned into the conv1 A operand P: per y1 position 32 bf16 =
//     [x_hi (9 taps) | x_hi | x_lo | 0 (5)] with x = x_hi + x_lo split into two bf16 (x_lo = bf16(x - x_hi)),
//     fragment-major so every MFMA A read is one conflict-free 16-byte LDS read.  The conv1 weights are
//     prepared as [w_hi | w_lo | w_hi | 0]: ONE v_mfma_f32_16x16x32_bf16 per 16 y1 positions x 16
//     channels gives conv1 with ~2^-16 relative error (x_hi w_hi + x_hi w_lo + x_lo w_hi; x_lo w_lo is
//     2^-18) in f32 accumulation -- y1 is then rounded to bf16 like the unfused path's y1;
//   then per chunk of 32 input channels: conv1 of the chunk for the (2R+1) x 41 y1 positions the output
//     rows need (incl. the conv2 zero padding column / rows) -> bias, ReLU, len1 mask -> bf16 y1 chunk in
//     LDS ([row][41 cols][40] bf16: the stride-2 A reads of a 16-position tile hit 16 distinct 4-bank
//     groups); then the 9 taps of conv2 over the chunk, one 16x16x32 MFMA per (16 positions, 16 output
//     channels, tap): A = y1 at the tap-shifted position (LDS), B = the tap's [co][32 ci] weight slab
//     read straight from L2 (16 bytes per lane, prefetched one tap ahead; 0.6 MB of bf16 weights per
//     encoder stay L2-resident);
//   epilogue: bias, ReLU, len2 mask, f32 output rows (b, t2, f2) x C -- the layout the following
//     Linear(C*F2 -> d) consumes.
// With `y1` given (the trained student: the backward needs y1's sign and its conv2 weight-gradient
// columns) the workgroup also writes the y1 rows it owns (t1 in [2 t2a, 2 t2a + 2R)) as bf16.
#include "gemm_common.h"

// timing probe points (tools/ss_probe.hip defines KPROBE; empty in the library)
#ifndef KPROBE
#define KPROBE(i)
#endif

namespace kdfm {
namespace {

constexpr int FS_NT = 512;   // 8 waves
constexpr int FS_CK = 32;    // input channels per chunk: the K of one 16x16x32 MFMA per tap
constexpr int FS_CKP = 40;   // y1 LDS position stride (bf16)
constexpr int FS_F1C = 41;   // y1 LDS columns: f1 = -1 (conv2 zero padding) .. 39
constexpr int FS_F2 = 20;    // output columns (F = 80 mel bins)
constexpr int FS_MC = 82;    // mel patch columns: f = -1 .. 80

struct FsArgs {
  const float* mel;            // (B, Tm, F) f32
  const int64_t* mel_len;      // frames >= mel_len read as 0 (NULL: none)
  const int64_t* len1;         // y1 rows >= len1 are 0 (NULL: none)
  const int64_t* len2;         // output rows >= len2 are 0 (NULL: none)
  const uint16_t* w1p;         // conv1 B operand [NCH*32 channels][32] bf16: [w_hi(9) | w_lo(9) | w_hi(9) | 0(5)]
  const float* b0;
  const uint16_t* w2p;         // conv2 B operand [9 taps][NCH chunks][NPAD co][32 ci] bf16
  const float* b2;
  float* y2;                   // (B*T2*F2, C) f32
  uint16_t* y1;                // optional (B*T1*F1, ldy1) bf16, channels [C, ldy1) written as zeros
  int B, Tm, F, T1, F1, T2, F2;
  int ldy1;                    // y1 row stride (elements): C <= ldy1 <= NCH * 32, a multiple of 8
};

__device__ __forceinline__ float bf_round(float x) { return (float)(__bf16)x; }

// C channels, R output rows per workgroup, WM x WN waves over (positions, output channels), MT x NT
// 16x16 tiles per wave
template <int C, int R, int WM, int WN, int MT, int NT>
__global__ __launch_bounds__(FS_NT, 1) void ss_fused_kernel(FsArgs a) {
  constexpr int NCH = (C + FS_CK - 1) / FS_CK;
  constexpr int NPAD = NT * 16 * WN;
  static_assert(NPAD >= C && WM * WN == 8, "wave grid");
  constexpr int NR1 = 2 * R + 1;                  // y1 rows of the patch
  constexpr int NQ = NR1 * FS_F1C;                // y1 positions
  constexpr int NPT = (NQ + 15) / 16;             // conv1 position tiles
  constexpr int MROWS = FS_F2 * R;                // output positions of the workgroup
  constexpr int MR = 4 * R + 3;                   // mel patch rows
  constexpr int Y1_BYTES = ((NPT * 16 * FS_CKP * 2 + 1023) / 1024) * 1024;
  static_assert(MR * FS_MC * 4 <= Y1_BYTES, "mel patch aliases the y1 buffer");
  // the chunk's conv2 weight slab ([9 taps][NPAD co][32 ci] bf16) staged in LDS when it fits beside y1 and P:
  // the B fragments are then LDS reads instead of L2 loads one tap ahead (an L2 round trip per tap)
  constexpr int WS_BYTES = 9 * NPAD * FS_CK * 2;
  constexpr bool STAGEB = Y1_BYTES + NPT * 1024 + WS_BYTES <= 160 * 1024;
  constexpr int WSU = WS_BYTES / 16;                       // 16-byte units of one slab
  constexpr int WSPT = STAGEB ? (WSU + FS_NT - 1) / FS_NT : 1;   // units per thread
  extern __shared__ __attribute__((aligned(16))) unsigned char fs_lds[];
  uint16_t* y1s = reinterpret_cast<uint16_t*>(fs_lds);
  float* mels = reinterpret_cast<float*>(fs_lds);
  unsigned char* Ps = fs_lds + Y1_BYTES;
  uint16_t* Wsl = reinterpret_cast<uint16_t*>(fs_lds + Y1_BYTES + NPT * 1024);

  KPROBE(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  const int nstrip = (a.T2 + R - 1) / R;
  const int b = (int)blockIdx.x / nstrip, s = (int)blockIdx.x - ((int)blockIdx.x / nstrip) * nstrip;
  const int t2a = s * R;
  const int t1a = 2 * t2a - 1;                    // y1 row of patch row 0
  const int tm0 = 2 * t1a - 1;                    // mel row of mel patch row 0
  const int ml = a.mel_len ? (int)min((int64_t)a.Tm, a.mel_len[b]) : a.Tm;
  const int l1 = a.len1 ? (int)min((int64_t)a.T1, a.len1[b]) : a.T1;
  const int l2 = a.len2 ? (int)min((int64_t)a.T2, a.len2[b]) : a.T2;

  // ---- prologue: mel patch, then the conv1 A operand P (fragment-major [tile][kq][r][8])
  const float* melb = a.mel + (int64_t)b * a.Tm * a.F;
  {
    // every load of the patch in flight at once: clamped (always valid) addresses, masked by a multiply
    // (a conditional load is branched around and waited for one by one)
    constexpr int MPT = (MR * FS_MC + FS_NT - 1) / FS_NT;
    float mv[MPT], mm[MPT];
#pragma unroll
    for (int u = 0; u < MPT; ++u) {
      const int e = threadIdx.x + u * FS_NT;
      const int i = e / FS_MC, j = e - i * FS_MC;
      const int t = tm0 + i, f = j - 1;
      const bool ok = e < MR * FS_MC && t >= 0 && t < ml && f >= 0 && f < a.F;
      mv[u] = melb[ok ? (int64_t)t * a.F + f : 0];
      mm[u] = ok ? 1.f : 0.f;
    }
#pragma unroll
    for (int u = 0; u < MPT; ++u) {
      const int e = threadIdx.x + u * FS_NT;
      if (e < MR * FS_MC) mels[e] = mv[u] * mm[u];
    }
  }
  __syncthreads();
  KPROBE(1);
  for (int q = threadIdx.x; q < NPT * 16; q += FS_NT) {
    const int i = q / FS_F1C, j = q - (q / FS_F1C) * FS_F1C;
    const bool in = q < NQ;
    float e[32];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int ky = k / 3, kx = k - (k / 3) * 3;
      const int col = max(0, 2 * j - 2 + kx);     // j = 0 is the padding column (its y1 is masked)
      const float x = in ? mels[(2 * i + ky) * FS_MC + col] : 0.f;
      const float hi = bf_round(x);
      e[k] = hi;
      e[9 + k] = hi;
      e[18 + k] = x - hi;                         // rounded to bf16 by the pack below
    }
#pragma unroll
    for (int k = 27; k < 32; ++k) e[k] = 0.f;
    const int pt = q >> 4, r = q & 15;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<bf16x8*>(Ps + ((pt * 4 + g) * 16 + r) * 16) = pack_bf16x8<bf16x8>(e + 8 * g);
  }
  __syncthreads();   // P complete; the mel patch (aliasing y1s) is dead from here
  KPROBE(2);

  // ---- conv2 geometry of this lane: the y1 element offset of its A row in every M tile
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  int yoff[MT];
  bool mvalid[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int mt = wm * MT + i;
    mvalid[i] = mt * 16 < MROWS;                  // wave-uniform
    const int p = mt * 16 + r16;
    const int t2l = p / FS_F2, f2 = p - (p / FS_F2) * FS_F2;
    yoff[i] = (p < MROWS) ? ((2 * t2l) * FS_F1C + 2 * f2) * FS_CKP + 8 * kq : 8 * kq;
  }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint16_t* w2l = a.w2p + (int64_t)((wn * NT) * 16 + r16) * FS_CK + 8 * kq;   // + ((tap*NCH + c)*NPAD + 16 j)*32

#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    // conv1 operands of the chunk: weight fragments (channels as the A rows) and this lane's 4 channels'
    // biases per 16-channel tile -- loaded before the slab so waiting for them does not wait for it
    const bf16x8 w1f0 = *reinterpret_cast<const bf16x8*>(a.w1p + (int64_t)(c * FS_CK + r16) * FS_CK + 8 * kq);
    const bf16x8 w1f1 = *reinterpret_cast<const bf16x8*>(a.w1p + (int64_t)(c * FS_CK + 16 + r16) * FS_CK + 8 * kq);
    float bias[2][4], chm[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ch = c * FS_CK + nt * 16 + 4 * kq + e;
        bias[nt][e] = a.b0[ch < C ? ch : 0];
        chm[nt][e] = ch < C ? 1.f : 0.f;
      }
    // the chunk's conv2 weight slab into registers first: its loads fly while conv1 runs
    uint4 wreg[WSPT];
    if constexpr (STAGEB) {
#pragma unroll
      for (int i = 0; i < WSPT; ++i) {
        const int u = threadIdx.x + i * FS_NT;
        const int uu = u < WSU ? u : 0;
        const int tap = uu / (NPAD * 4), rest = uu - tap * (NPAD * 4);
        wreg[i] = *reinterpret_cast<const uint4*>(a.w2p + ((int64_t)(tap * NCH + c) * NPAD * FS_CK + rest * 8));
      }
    }
    // ---- conv1 of channels [32c, 32c + 32) for every y1 position of the patch -> bf16 y1 chunk in LDS.
    // Computed transposed (channels x positions: A = the weights, B = the patch operand), so a lane holds
    // 4 consecutive channels of ONE position: one validity test and one 8-byte LDS store per tile
    for (int pt = wave; pt < NPT; pt += 8) {
      const bf16x8 pf = *reinterpret_cast<const bf16x8*>(Ps + ((pt * 4 + kq) * 16 + r16) * 16);
      const f32x4 v0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f0, pf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const f32x4 v1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f1, pf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const int q = pt * 16 + r16;
      const int i = q / FS_F1C, j = q - i * FS_F1C;
      const int t1 = t1a + i;
      const float pm = (q < NQ && t1 >= 0 && t1 < l1 && j >= 1) ? 1.f : 0.f;
      float y[2][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[0][e] = fmaxf(v0[e] + bias[0][e], 0.f) * (pm * chm[0][e]);
        y[1][e] = fmaxf(v1[e] + bias[1][e], 0.f) * (pm * chm[1][e]);
      }
      if (q < NPT * 16) {
        uint16_t* dst = y1s + q * FS_CKP + 4 * kq;
        *reinterpret_cast<uint2*>(dst) = make_uint2(pack_bf16x2(y[0][0], y[0][1]), pack_bf16x2(y[0][2], y[0][3]));
        *reinterpret_cast<uint2*>(dst + 16) = make_uint2(pack_bf16x2(y[1][0], y[1][1]), pack_bf16x2(y[1][2], y[1][3]));
      }
    }
    if (c < 8) KPROBE(3 + 3 * c);
    if constexpr (STAGEB) {
#pragma unroll
      for (int i = 0; i < WSPT; ++i) {
        const int u = threadIdx.x + i * FS_NT;
        if (u < WSU) *reinterpret_cast<uint4*>(Wsl + u * 8) = wreg[i];
      }
    }
    __syncthreads();
    if (c < 8) KPROBE(4 + 3 * c);
    if (a.y1) {
      // the y1 rows this workgroup owns (patch rows 1 .. 2R), 8 channels per 16-byte store
      constexpr int UN = 2 * R * 40 * 4;
      for (int u = threadIdx.x; u < UN; u += FS_NT) {
        const int g = u & 3, pos = u >> 2;
        const int i = 1 + pos / 40, f1 = pos - (pos / 40) * 40;
        const int t1 = t1a + i, ch = c * FS_CK + 8 * g;
        if (t1 < a.T1 && ch < a.ldy1)
          *reinterpret_cast<bf16x8*>(a.y1 + (((int64_t)b * a.T1 + t1) * a.F1 + f1) * a.ldy1 + ch) =
              *reinterpret_cast<const bf16x8*>(y1s + (i * FS_F1C + f1 + 1) * FS_CKP + 8 * g);
      }
    }
    // ---- conv2 over the chunk: 9 taps, B slabs from the LDS image (STAGEB) or from L2 one tap ahead
    if constexpr (STAGEB) {
      const uint16_t* wl = Wsl + ((wn * NT) * 16 + r16) * FS_CK + 8 * kq;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        bf16x8 bl[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) bl[j] = *reinterpret_cast<const bf16x8*>(wl + (tap * NPAD + j * 16) * FS_CK);
        const int toff = ((tap / 3) * FS_F1C + (tap % 3)) * FS_CKP;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          if (!mvalid[i]) continue;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(y1s + yoff[i] + toff);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bl[j], acc[i][j], 0, 0, 0);
        }
      }
      if (c < 8) KPROBE(5 + 3 * c);
      __syncthreads();   // the next chunk's conv1 overwrites y1s (and its slab Wsl)
      continue;
    }
    bf16x8 bq[2][NT];
    const uint16_t* wc = w2l + (int64_t)c * NPAD * FS_CK;
#pragma unroll
    for (int j = 0; j < NT; ++j) bq[0][j] = *reinterpret_cast<const bf16x8*>(wc + (int64_t)j * 16 * FS_CK);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) {
        const uint16_t* wt = wc + (int64_t)(tap + 1) * NCH * NPAD * FS_CK;
#pragma unroll
        for (int j = 0; j < NT; ++j) bq[(tap + 1) & 1][j] = *reinterpret_cast<const bf16x8*>(wt + (int64_t)j * 16 * FS_CK);
      }
      const int toff = ((tap / 3) * FS_F1C + (tap % 3)) * FS_CKP;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (!mvalid[i]) continue;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(y1s + yoff[i] + toff);
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bq[tap & 1][j], acc[i][j], 0, 0, 0);
      }
    }
    if (c < 8) KPROBE(5 + 3 * c);
    __syncthreads();   // the next chunk's conv1 overwrites y1s
  }
  KPROBE(30);

  // ---- epilogue: bias + ReLU + len2 mask, f32 rows (b, t2, f2) x C.  The workgroup's output rows are ONE
  // contiguous range of y2 (utterance b, rows t2a .. t2a + R - 1, all 20 columns, all C channels): the tile goes
  // through LDS (dead after the last chunk's barrier) and leaves as 16-byte stores over that range, whole
  // 64-byte segments, instead of the accumulators' 64-byte column runs (a 352-byte row at C = 88 puts half of
  // those across two segments)
  float* ys = reinterpret_cast<float*>(fs_lds);   // [MROWS][C]
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = (wn * NT + j) * 16 + r16;
    const float bn = n < C ? a.b2[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = (wm * MT + i) * 16 + 4 * kq + e;
        const int t2 = t2a + p / FS_F2;
        if (p < MROWS && n < C) {
          const float v = fmaxf(acc[i][j][e] + bn, 0.f);
          ys[p * C + n] = t2 < l2 ? v : 0.f;
        }
      }
    }
  }
  __syncthreads();
  {
    const int nr = min(R, a.T2 - t2a) * FS_F2;   // rows of this workgroup inside the utterance
    const int n4 = nr * C / 4;
    float4* dst = reinterpret_cast<float4*>(a.y2 + ((int64_t)b * a.T2 + t2a) * a.F2 * C);
    const float4* src = reinterpret_cast<const float4*>(ys);
    for (int u = threadIdx.x; u < n4; u += FS_NT) dst[u] = src[u];
  }
  KPROBE(31);
}

template <int C, int R, int WM, int WN, int MT, int NT>
int fs_launch(const FsArgs& a, hipStream_t st) {
  constexpr int NR1 = 2 * R + 1, NQ = NR1 * FS_F1C, NPT = (NQ + 15) / 16;
  constexpr int Y1_BYTES = ((NPT * 16 * FS_CKP * 2 + 1023) / 1024) * 1024;
  constexpr int NPAD = NT * 16 * WN, WS_BYTES = 9 * NPAD * FS_CK * 2;
  constexpr size_t base = (size_t)Y1_BYTES + (size_t)NPT * 1024;
  constexpr size_t lds0 = base + (base + WS_BYTES <= 160 * 1024 ? (size_t)WS_BYTES : 0);   // STAGEB (kernel)
  constexpr size_t Y2_BYTES = (size_t)FS_F2 * R * C * 4;   // the epilogue's output tile
  constexpr size_t lds = lds0 > Y2_BYTES ? lds0 : Y2_BYTES;
  static_assert(lds <= 160 * 1024, "LDS");
  static bool once = [] {
    (void)hipFuncSetAttribute((const void*)ss_fused_kernel<C, R, WM, WN, MT, NT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)once;
  const int nstrip = (a.T2 + R - 1) / R;
  hipLaunchKernelGGL((ss_fused_kernel<C, R, WM, WN, MT, NT>), dim3((unsigned)(a.B * nstrip)), dim3(FS_NT), lds, st, a);
  return check_launch("kdfm_subsample_fused");
}

// conv1 operand [NCH*32][32]: rows = channels (zero past C); conv2 operand [9][NCH][npad][32]
__global__ __launch_bounds__(256) void fs_wprep_kernel(const float* __restrict__ w0, const float* __restrict__ w2,
                                                       uint16_t* __restrict__ w1p, uint16_t* __restrict__ w2p, int C,
                                                       int nch, int npad) {
  const int64_t n1 = (int64_t)nch * 32 * 32;
  const int64_t n2 = (int64_t)9 * nch * npad * 32;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx < n1) {
    const int ch = (int)(idx / 32), k = (int)(idx % 32);
    float v = 0.f;
    if (ch < C && k < 27) {
      const float w = w0[ch * 9 + (k % 9)];
      const float hi = bf_round(w);
      v = (k >= 9 && k < 18) ? w - hi : hi;
    }
    w1p[idx] = f2bf(v);
  } else if (idx < n1 + n2) {
    const int64_t e = idx - n1;
    const int k = (int)(e % 32);
    const int co = (int)((e / 32) % npad);
    const int c = (int)((e / (32 * (int64_t)npad)) % nch);
    const int tap = (int)(e / (32 * (int64_t)npad * nch));
    const int ci = c * 32 + k;
    w2p[e] = f2bf((co < C && ci < C) ? w2[((int64_t)co * C + ci) * 9 + tap] : 0.f);
  }
}

int fs_config(int64_t C, int& nch, int& npad) {
  if (C == 176 || C == 192) { nch = (int)ceil_div(C, 32); npad = 192; return 1; }
  if (C == 88 || C == 96) { nch = 3; npad = 96; return 1; }
  return 0;
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_subsample_fused_supported(int64_t C, int64_t F) {
  int nch, npad;
  return F == 80 && kdfm::fs_config(C, nch, npad);
}

int64_t kdfm_subsample_fused_wprep_elems(int64_t C) {
  int nch, npad;
  if (!kdfm::fs_config(C, nch, npad)) return 0;
  return (int64_t)nch * 32 * 32 + (int64_t)9 * nch * npad * 32;
}

int kdfm_subsample_fused_wprep(const float* w0, const float* w2, uint16_t* wp, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(w0 && w2 && wp, "null pointer");
  int nch, npad;
  if (!fs_config(C, nch, npad)) {
    set_error("kdfm_subsample_fused_wprep: unsupported channel count");
    return KDFM_EUNSUPPORTED;
  }
  const int64_t n1 = (int64_t)nch * 32 * 32;
  const int64_t n = n1 + (int64_t)9 * nch * npad * 32;
  hipLaunchKernelGGL(fs_wprep_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), w0, w2, wp,
                     wp + n1, (int)C, nch, npad);
  return check_launch("kdfm_subsample_fused_wprep");
}

int kdfm_subsample_fused(const float* mel, const int64_t* mel_len, const int64_t* len1, const int64_t* len2,
                         const uint16_t* wp, const float* b0, const float* b2, float* y2, uint16_t* y1, int64_t B,
                         int64_t Tm, int64_t F, int64_t C, int64_t ldy1, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(mel && wp && b0 && b2 && y2, "null pointer");
  int nch, npad;
  KDFM_REQUIRE(F == 80 && fs_config(C, nch, npad), "unsupported shape (F = 80, C in {88, 96, 176, 192})");
  KDFM_REQUIRE(B > 0 && Tm > 0, "empty batch");
  KDFM_REQUIRE(((((uintptr_t)wp) | ((uintptr_t)y1) | ((uintptr_t)y2)) & 15) == 0, "wp / y1 / y2 must be 16-byte aligned");
  KDFM_REQUIRE(y1 == nullptr || (ldy1 >= C && ldy1 <= nch * 32 && ldy1 % 8 == 0),
               "ldy1 must be a multiple of 8 in [C, 32 * ceil(C / 32)]");
  FsArgs a;
  a.mel = mel; a.mel_len = mel_len; a.len1 = len1; a.len2 = len2;
  a.w1p = wp; a.b0 = b0; a.w2p = wp + (int64_t)nch * 32 * 32; a.b2 = b2; a.y2 = y2; a.y1 = y1;
  a.B = (int)B; a.Tm = (int)Tm; a.F = (int)F;
  a.T1 = (int)((Tm - 1) / 2 + 1); a.F1 = (int)((F - 1) / 2 + 1);
  a.T2 = (a.T1 - 1) / 2 + 1; a.F2 = (a.F1 - 1) / 2 + 1;
  a.ldy1 = (int)(y1 ? ldy1 : C);
  KDFM_REQUIRE(a.F2 == FS_F2, "F2 must be 20");
  hipStream_t st = as_stream(stream);
  switch (C) {
    case 176: return fs_launch<176, 8, 2, 4, 5, 3>(a, st);   // Conformer-CTC-small teacher
    case 192: return fs_launch<192, 8, 2, 4, 5, 3>(a, st);
    case 88: return fs_launch<88, 8, 4, 2, 3, 3>(a, st);     // the halved student
    default: return fs_launch<96, 8, 4, 2, 3, 3>(a, st);
  }
}

}  // extern "C"
