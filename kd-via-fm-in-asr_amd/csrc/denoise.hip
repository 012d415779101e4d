// Fused SimpleDenoiser chain of the KD heads (bf16 MFMA, f32 state): all S steps of
//   x <- x - net(x) / S,   net = Conv1d(L, L, 3, pad 1) -> ReLU -> Conv1d(L, L, 3, pad 1)
// (asr_train_diffm.py:444-460; S = 9 for ver5, called at :685-724) in one launch forward and one
// launch for the data-gradient backward, over the stacked (16 layers x B) utterances of T frames
// (kdfm/heads.py).  The unfused path ran two conv launches per step, each reading and writing a
// 205k x 96 f32 tensor (~1.5 ms forward, ~1.3 ms backward per step at the bench shape).
//
// Decomposition.  The conv couples neighbouring frames, so a workgroup owns a WINDOW of frames of
// one utterance and keeps its activation image in LDS across all 2S convs.  A window ends either at
// the utterance edge (true zero padding) or inside the utterance; there each conv spreads the unknown
// frame beyond the edge one frame further in, so a window carries H = 2S halo frames per interior
// edge and writes only its VALID frames.  At the bench shape (T = 401, S = 9) that is two windows of
// ~219 frames per utterance (9% recomputed).  LDS: both conv weight images (bf16, [out][tap*L + in],
// 2 x 56.8 KB) + the activation image (bf16, [frame][L], <= 222 rows x 208 B) + biases.
//
// Each conv is C^T (L outputs x 64 frames per wave) = Wimg (L x 3L) x Ximg^T with
// v_mfma_f32_32x32x16_bf16: A = a weight-image row (16 B), B = an image row shifted by the tap
// (16 B); the accumulator gives lane (r, h) frame r of its 32-frame tile and outputs
// 32 mt + 8 q + 4 h + 0..3, so writing an activation back into the image is one 8-byte LDS store
// per 4 outputs.  Per step:  conv1 -> a = relu(. + b1) -> image;  conv2 -> x -= (. + b2) / S ->
// image.  Saved for the backward and the weight gradients (bf16, (S, n, L)): X[i] = x_i (conv1's
// input) and A[i] = a_i (conv2's input and the ReLU mask) — exactly the values the bf16 GEMM path
// rounds at staging.
//
// Backward (g = dL/dx_S in):  for i = S-1..0:  GV[i] = g;  da = -(1/S) conv2^T(g) . [a_i > 0];
// DA[i] = da;  g += conv1^T(da).  conv^T is the same kernel body on the transposed weight images
// [in][tap'*L + out] = W[out][in][2 - tap'].  The weight gradients are then two row-parallel CONV
// launches over the stacked (S n) rows (kdfm_wgrad_bf16_conv): dW1 += DA (x) X, dW2 += -(1/S) GV (x) A.
#include "gemm_common.h"

namespace kdfm {
namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T* lds_at(uint16_t* base, int off) {
  return reinterpret_cast<__attribute__((address_space(3))) T*>((lds_u16*)base + off);
}

constexpr int DN_L = 96;                    // latent width (features)
constexpr int DN_K = 3 * DN_L;              // contraction length of one conv (tap, in)
constexpr int DN_LDW = DN_K + 8;            // weight image row stride (bf16): 592 B
constexpr int DN_LDX = DN_L + 8;            // activation image row stride (bf16): 208 B
constexpr int DN_NT = 256;                  // 4 waves x 64 frames
constexpr int DN_WMAX = 220;                // frames per window (image rows: + 2 edge rows)
constexpr int DN_WIMG = DN_L * DN_LDW;      // elements of one weight image
constexpr int DN_XROWS = DN_WMAX + 2;
constexpr int DN_OFF_X = 2 * DN_WIMG;                       // activation image
constexpr int DN_OFF_B = DN_OFF_X + DN_XROWS * DN_LDX;      // biases (f32, as uint16 pairs)
constexpr size_t DN_LDS = (size_t)(DN_OFF_B + 2 * 2 * DN_L) * sizeof(uint16_t);

__device__ __forceinline__ uint32_t pk2(float a, float b) { return pack_bf16x2(a, b); }
__device__ __forceinline__ float bf2f(uint32_t b16) { return __builtin_bit_cast(float, b16 << 16); }

struct DnGeo {
  int64_t T;       // frames per utterance
  int P;           // windows per utterance
  int V;           // valid frames per window (the last one may have fewer)
  int H;           // halo frames per interior edge (2 S)
};

// window of block b: utterance u, frames [ws, we), valid frames [vs, ve)
struct DnWin {
  int64_t u;
  int ws, we, vs, ve;
};
__device__ __forceinline__ DnWin dn_window(const DnGeo& g, int64_t wid) {
  DnWin w;
  w.u = wid / g.P;
  const int p = (int)(wid - w.u * g.P);
  const int T = (int)g.T;
  w.vs = p * g.V;
  w.ve = min(T, w.vs + g.V);
  w.ws = max(0, w.vs - g.H);
  w.we = min(T, w.ve + g.H);
  return w;
}

// weight images [o][tap*L + i] = bf16(W[o][i][tap]) (fwd) or [i][tap*L + o] = bf16(W[o][i][2 - tap]) (bwd)
// for both convs, in the exact LDS layout (pad columns zero); W is PyTorch's Conv1d weight (L, L, 3).
// Built once per call by dn_wprep_kernel; every persistent workgroup copies it with 16-byte loads.
constexpr int DN_WCHUNKS = 2 * DN_WIMG / 8;   // 16-byte chunks of both images
__global__ __launch_bounds__(256) void dn_wprep_kernel(const float* __restrict__ W1, const float* __restrict__ W2,
                                                       uint16_t* __restrict__ wimg, int bwd) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * DN_WIMG) return;
  const int which = e / DN_WIMG, q = e - which * DN_WIMG;
  const int row = q / DN_LDW, k = q - row * DN_LDW;
  float v = 0.f;
  if (k < DN_K) {
    const float* W = which ? W2 : W1;
    const int tap = k / DN_L, col = k - tap * DN_L;
    v = bwd ? W[((int64_t)col * DN_L + row) * 3 + (2 - tap)] : W[((int64_t)row * DN_L + col) * 3 + tap];
  }
  wimg[e] = f2bf(v);
}

__device__ __forceinline__ void dn_load_w(uint16_t* lds, const uint16_t* __restrict__ wimg) {
  constexpr int PER = (DN_WCHUNKS + DN_NT - 1) / DN_NT;
  bf16x8 v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = j * DN_NT + threadIdx.x;
    if (e < DN_WCHUNKS) v[j] = *reinterpret_cast<const bf16x8*>(wimg + 8 * e);
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = j * DN_NT + threadIdx.x;
    if (e < DN_WCHUNKS) *lds_at<bf16x8>(lds, 8 * e) = v[j];
  }
}

// acc[nt][mt][i] = sum_{tap, c} Wimg[32 mt + f(i)][tap*L + c] * Ximg[lr(nt) + tap][c]
// (image row j holds window frame j - 1); rows of garbage tiles are clamped into the image and
// computed like real ones (a wave's time is set by its slowest tile anyway).  Software-pipelined:
// the 5 fragments of k-step ks+1 are read from LDS while the 6 MFMAs of ks run.
struct DnFrag {
  bf16x8 b[2], a[3];
};
__device__ __forceinline__ void dn_frag(DnFrag& f, uint16_t* lds, int img, int xr0, int xr1, int wr, int ks) {
  const int tap = ks / (DN_L / 16), kc = ks - tap * (DN_L / 16);
  f.b[0] = *lds_at<bf16x8>(lds, xr0 + tap * DN_LDX + kc * 16);
  f.b[1] = *lds_at<bf16x8>(lds, xr1 + tap * DN_LDX + kc * 16);
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) f.a[mt] = *lds_at<bf16x8>(lds, img + wr + mt * 32 * DN_LDW + ks * 16);
}
__device__ __forceinline__ void dn_conv(f32x16 (&acc)[2][3], uint16_t* lds, int img, int wave, int lane, int nrows) {
  const int r = lane & 31, h = lane >> 5;
  // image rows of tap 0 (clamped so taps 1, 2 stay inside the image: garbage rows only)
  const int lr0 = min(wave * 64 + r, nrows - 1), lr1 = min(wave * 64 + 32 + r, nrows - 1);
  const int xr0 = DN_OFF_X + lr0 * DN_LDX + 8 * h, xr1 = DN_OFF_X + lr1 * DN_LDX + 8 * h;
  const int wr = r * DN_LDW + 8 * h;
  constexpr int KS = DN_K / 16;
  DnFrag f[2];
  dn_frag(f[0], lds, img, xr0, xr1, wr, 0);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 1 < KS) dn_frag(f[(ks + 1) & 1], lds, img, xr0, xr1, wr, ks + 1);
    const DnFrag& c = f[ks & 1];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        if (ks == 0) {
          f32x16 z;
#pragma unroll
          for (int i = 0; i < 16; ++i) z[i] = 0.f;
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c.a[mt], c.b[nt], z, 0, 0, 0);
        } else {
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c.a[mt], c.b[nt], acc[nt][mt], 0, 0, 0);
        }
      }
  }
}

// the wave's 2 x 32 frames x 96 outputs packed to bf16 pairs once (one v_cvt_pk_bf16_f32 per pair),
// then written to the LDS image and, for the saves, to HBM
typedef uint32_t DnPk[2][3][8];
template <typename V>
__device__ __forceinline__ void dn_pack(DnPk& p, const V& v) {
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < 8; ++j) p[nt][mt][j] = pk2(v[nt][mt][2 * j], v[nt][mt][2 * j + 1]);
}

// image row (lr + 1) <- the packed values, for the wave's real frames (lr < nrows)
__device__ __forceinline__ void dn_put(uint16_t* lds, const DnPk& p, int wave, int lane, int nrows) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int lr = wave * 64 + nt * 32 + r;
    if (lr >= nrows) continue;
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *lds_at<u32x2>(lds, DN_OFF_X + (lr + 1) * DN_LDX + mt * 32 + 8 * q + 4 * h) =
            u32x2{p[nt][mt][2 * q], p[nt][mt][2 * q + 1]};
  }
}

// save the image's valid frames [f_lo, f_hi) (window-relative) to dst rows row0 + f: coalesced
// 16-byte chunks read back from LDS after the barrier that completed the image (row-per-lane 8-byte
// stores straight from the accumulator layout are store-issue bound: 24 per lane per save)
__device__ __forceinline__ void dn_save(uint16_t* __restrict__ dst, const uint16_t* lds, int64_t row0, int f_lo,
                                        int f_hi) {
  constexpr int CPR = DN_L / 8;   // 16-byte chunks per row
  const int chunks = (f_hi - f_lo) * CPR;
  for (int e = threadIdx.x; e < chunks; e += DN_NT) {
    const int f = f_lo + e / CPR, c = (e % CPR) * 8;
    const bf16x8 v = *lds_at<bf16x8>(const_cast<uint16_t*>(lds), DN_OFF_X + (f + 1) * DN_LDX + c);
    *reinterpret_cast<bf16x8*>(dst + (row0 + f) * DN_L + c) = v;
  }
}

// global row-major (rows x L) f32 stores / loads of the wave's frames (stores restricted to [f_lo, f_hi))
template <typename V>
__device__ __forceinline__ void dn_store_f32(float* __restrict__ dst, const V& v, int64_t row0, int wave, int lane,
                                             int f_lo, int f_hi) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int lr = wave * 64 + nt * 32 + r;
    if (lr < f_lo || lr >= f_hi) continue;
    float* base = dst + (row0 + lr) * DN_L;
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(base + mt * 32 + 8 * q + 4 * h) =
            make_float4(v[nt][mt][4 * q], v[nt][mt][4 * q + 1], v[nt][mt][4 * q + 2], v[nt][mt][4 * q + 3]);
  }
}
template <typename V>
__device__ __forceinline__ void dn_load_f32(V& v, const float* __restrict__ src, int64_t row0, int wave, int lane,
                                            int nrows) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int lr = wave * 64 + nt * 32 + r;
    const bool ok = lr < nrows;
    const float* base = src + (row0 + (ok ? lr : 0)) * DN_L;
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 t = *reinterpret_cast<const float4*>(base + mt * 32 + 8 * q + 4 * h);
        v[nt][mt][4 * q] = ok ? t.x : 0.f;
        v[nt][mt][4 * q + 1] = ok ? t.y : 0.f;
        v[nt][mt][4 * q + 2] = ok ? t.z : 0.f;
        v[nt][mt][4 * q + 3] = ok ? t.w : 0.f;
      }
  }
}

// zero the window's two edge rows (frames ws-1 and we: true zero padding at an utterance edge, or
// the halo's unknown frame); rows past nrows + 1 are never read (dn_conv clamps into the image)
__device__ __forceinline__ void dn_zero_edges(uint16_t* lds, int nrows) {
  for (int e = threadIdx.x; e < 2 * DN_LDX / 8; e += DN_NT) {
    const int row = e < DN_LDX / 8 ? 0 : nrows + 1, c = (e % (DN_LDX / 8)) * 8;
    bf16x8 z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = 0;
    *lds_at<bf16x8>(lds, DN_OFF_X + row * DN_LDX + c) = z;
  }
}

struct DnFwd {
  const float* z; const uint16_t* wimg; const float* b1; const float* b2;
  uint16_t* X; uint16_t* A; float* out;
  int64_t n, nwin; int S;
};

// persistent: each workgroup stages the weight images once and walks windows wid = blockIdx.x,
// blockIdx.x + gridDim.x, ... (every barrier is reached by all waves of the workgroup)
__global__ __launch_bounds__(DN_NT, 1) void denoise_fwd_kernel(DnFwd a, DnGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t dn_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int64_t nL = a.n * DN_L;
  dn_load_w(dn_lds, a.wimg);
  for (int e = threadIdx.x; e < 2 * DN_L; e += DN_NT)
    *lds_at<float>(dn_lds, DN_OFF_B + 2 * e) = e < DN_L ? a.b1[e] : a.b2[e - DN_L];
  auto bias4 = [&](int which, int mt, int q) {
    return *lds_at<f32x4>(dn_lds, DN_OFF_B + 2 * (which * DN_L + mt * 32 + 8 * q + 4 * h));
  };
  const float invS = 1.f / (float)a.S;
  for (int64_t wid = blockIdx.x; wid < a.nwin; wid += gridDim.x) {
    const DnWin w = dn_window(g, wid);
    const int nrows = w.we - w.ws;
    const int f_lo = w.vs - w.ws, f_hi = w.ve - w.ws;   // valid frames, window-relative
    const int64_t row0 = w.u * g.T + w.ws;              // global row of window frame 0
    float x[2][3][16];
    f32x16 acc[2][3];
    dn_load_f32(x, a.z, row0, wave, lane, nrows);
    __syncthreads();   // weights staged / the previous window's last conv has read the image
    dn_zero_edges(dn_lds, nrows);
    {
      DnPk pk;
      dn_pack(pk, x);
      dn_put(dn_lds, pk, wave, lane, nrows);
    }
    __syncthreads();
    if (a.X) dn_save(a.X, dn_lds, row0, f_lo, f_hi);
    for (int i = 0; i < a.S; ++i) {
      dn_conv(acc, dn_lds, 0, wave, lane, nrows);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 b = bias4(0, mt, q);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[nt][mt][4 * q + k] = fmaxf(acc[nt][mt][4 * q + k] + b[k], 0.f);
          }
      __syncthreads();   // every wave has read the image
      {
        DnPk pk;
        dn_pack(pk, acc);
        dn_put(dn_lds, pk, wave, lane, nrows);
      }
      __syncthreads();
      if (a.A) dn_save(a.A + i * nL, dn_lds, row0, f_lo, f_hi);
      dn_conv(acc, dn_lds, DN_WIMG, wave, lane, nrows);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 b = bias4(1, mt, q);
#pragma unroll
            for (int k = 0; k < 4; ++k) x[nt][mt][4 * q + k] -= (acc[nt][mt][4 * q + k] + b[k]) * invS;
          }
      if (i + 1 < a.S) {
        __syncthreads();
        DnPk pk;
        dn_pack(pk, x);
        dn_put(dn_lds, pk, wave, lane, nrows);
        __syncthreads();
        if (a.X) dn_save(a.X + (i + 1) * nL, dn_lds, row0, f_lo, f_hi);
      }
    }
    dn_store_f32(a.out, x, row0, wave, lane, f_lo, f_hi);
  }
}

struct DnBwd {
  const float* gout; const uint16_t* A; const uint16_t* wimg;
  uint16_t* GV; uint16_t* DA; float* gin;
  int64_t n, nwin; int S;
};

__global__ __launch_bounds__(DN_NT, 1) void denoise_bwd_kernel(DnBwd a, DnGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t dn_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t nL = a.n * DN_L;
  dn_load_w(dn_lds, a.wimg);
  const float invS = 1.f / (float)a.S;
  for (int64_t wid = blockIdx.x; wid < a.nwin; wid += gridDim.x) {
    const DnWin w = dn_window(g, wid);
    const int nrows = w.we - w.ws;
    const int f_lo = w.vs - w.ws, f_hi = w.ve - w.ws;
    const int64_t row0 = w.u * g.T + w.ws;
    float gx[2][3][16];
    f32x16 acc[2][3];
    dn_load_f32(gx, a.gout, row0, wave, lane, nrows);
    __syncthreads();   // weights staged / the previous window's last conv has read the image
    dn_zero_edges(dn_lds, nrows);
    for (int i = a.S - 1; i >= 0; --i) {
      {
        DnPk pk;
        dn_pack(pk, gx);
        dn_put(dn_lds, pk, wave, lane, nrows);
      }
      __syncthreads();
      if (a.GV) dn_save(a.GV + i * nL, dn_lds, row0, f_lo, f_hi);
      // the ReLU mask of step i (saved forward activation), loaded before the conv so its latency hides
      uint2 msk[2][3][4];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int lr = wave * 64 + nt * 32 + r;
        const uint16_t* ai = a.A + i * nL + (row0 + (lr < nrows ? lr : 0)) * DN_L;
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int q = 0; q < 4; ++q) msk[nt][mt][q] = *reinterpret_cast<const uint2*>(ai + mt * 32 + 8 * q + 4 * h);
      }
      dn_conv(acc, dn_lds, DN_WIMG, wave, lane, nrows);
      // da = -(1/S) conv2^T(g) . [a_i > 0]
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const bool ok = wave * 64 + nt * 32 + r < nrows;
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint2 m = msk[nt][mt][q];
            const uint32_t e[4] = {m.x & 0xFFFFu, m.x >> 16, m.y & 0xFFFFu, m.y >> 16};
#pragma unroll
            for (int k = 0; k < 4; ++k)
              acc[nt][mt][4 * q + k] = (ok && bf2f(e[k]) > 0.f) ? -invS * acc[nt][mt][4 * q + k] : 0.f;
          }
      }
      __syncthreads();
      {
        DnPk pk;
        dn_pack(pk, acc);
        dn_put(dn_lds, pk, wave, lane, nrows);
      }
      __syncthreads();
      if (a.DA) dn_save(a.DA + i * nL, dn_lds, row0, f_lo, f_hi);
      dn_conv(acc, dn_lds, 0, wave, lane, nrows);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int k = 0; k < 16; ++k) gx[nt][mt][k] += acc[nt][mt][k];
      __syncthreads();
    }
    dn_store_f32(a.gin, gx, row0, wave, lane, f_lo, f_hi);
  }
}

// windows per utterance: the smallest P whose windows (valid span + halo per interior edge) fit
bool dn_geo(int64_t T, int S, DnGeo& g) {
  g.T = T;
  g.H = 2 * S;
  for (int P = 1; P <= 64; ++P) {
    const int V = (int)ceil_div(T, P);
    bool fits = true;
    for (int p = 0; p < P && fits; ++p) {
      const int vs = p * V, ve = (int)std::min<int64_t>(T, vs + V);
      if (vs >= ve) { fits = false; break; }
      const int ws = std::max(0, vs - g.H), we = (int)std::min<int64_t>(T, ve + g.H);
      fits = we - ws <= DN_WMAX;
    }
    if (fits) {
      g.P = P;
      g.V = V;
      return true;
    }
  }
  return false;
}

template <typename K>
void dn_allow_lds(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DN_LDS);
}

unsigned dn_grid(int64_t nwin) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount
                                                                                                  : 256;
  }
  return (unsigned)(nwin < cus ? nwin : cus);
}

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_denoise_wimg_elems(void) { return 2 * kdfm::DN_WIMG; }

int kdfm_denoise_chain_fwd(const float* z, const float* W1, const float* b1, const float* W2, const float* b2,
                           uint16_t* wimg, uint16_t* X, uint16_t* A, float* out, int64_t n, int64_t T, int32_t L,
                           int32_t S, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(z && W1 && b1 && W2 && b2 && wimg && out, "null pointer");
  KDFM_REQUIRE(L == DN_L, "the fused denoiser is compiled for latent width 96");
  KDFM_REQUIRE(S >= 1 && T >= 1 && n % T == 0, "bad steps / frames (rows must be whole utterances)");
  KDFM_REQUIRE(((((uintptr_t)z) | ((uintptr_t)out) | ((uintptr_t)X) | ((uintptr_t)A) | ((uintptr_t)wimg)) & 15) == 0,
               "row operands must be 16-byte aligned");
  if (n <= 0) return KDFM_OK;
  DnGeo g;
  KDFM_REQUIRE(dn_geo(T, S, g), "too many steps for the window size");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(dn_wprep_kernel, dim3((unsigned)ceil_div(2 * DN_WIMG, 256)), dim3(256), 0, st, W1, W2, wimg, 0);
  const int64_t nwin = (n / T) * g.P;
  DnFwd a{z, wimg, b1, b2, X, A, out, n, nwin, S};
  static bool once = (dn_allow_lds(denoise_fwd_kernel), true);
  (void)once;
  hipLaunchKernelGGL(denoise_fwd_kernel, dim3(dn_grid(nwin)), dim3(DN_NT), DN_LDS, st, a, g);
  return check_launch("kdfm_denoise_chain_fwd");
}

int kdfm_denoise_chain_bwd(const float* gout, const uint16_t* A, const float* W1, const float* W2, uint16_t* wimg,
                           uint16_t* GV, uint16_t* DA, float* gin, int64_t n, int64_t T, int32_t L, int32_t S,
                           void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(gout && A && W1 && W2 && wimg && gin, "null pointer");
  KDFM_REQUIRE(L == DN_L, "the fused denoiser is compiled for latent width 96");
  KDFM_REQUIRE(S >= 1 && T >= 1 && n % T == 0, "bad steps / frames (rows must be whole utterances)");
  KDFM_REQUIRE(((((uintptr_t)gout) | ((uintptr_t)A) | ((uintptr_t)GV) | ((uintptr_t)DA) | ((uintptr_t)gin) |
                 ((uintptr_t)wimg)) & 15) == 0, "row operands must be 16-byte aligned");
  if (n <= 0) return KDFM_OK;
  DnGeo g;
  KDFM_REQUIRE(dn_geo(T, S, g), "too many steps for the window size");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(dn_wprep_kernel, dim3((unsigned)ceil_div(2 * DN_WIMG, 256)), dim3(256), 0, st, W1, W2, wimg, 1);
  const int64_t nwin = (n / T) * g.P;
  DnBwd a{gout, A, wimg, GV, DA, gin, n, nwin, S};
  static bool once = (dn_allow_lds(denoise_bwd_kernel), true);
  (void)once;
  hipLaunchKernelGGL(denoise_bwd_kernel, dim3(dn_grid(nwin)), dim3(DN_NT), DN_LDS, st, a, g);
  return check_launch("kdfm_denoise_chain_bwd");
}

}  // extern "C"
