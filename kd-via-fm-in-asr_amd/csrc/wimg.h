// Fragment-major bf16 weight images of the LayerNorm-fused / row-streaming Conformer kernels (ffn.hip,
// lnproj.hip, rowgemm.hip): one lane-contiguous 1 KB block per (32-row tile, 16-wide k-step), lane
// (r = lane & 31, h = lane >> 5) holding the 8 k-consecutive values [32 tile + r][16 ks + 8 h + j].
// The per-fragment value functions are shared by the single-image prep kernels and by
// kdfm_wimg_prep_batch, which builds every image of a model in one launch per training step.
#pragma once
#include "common.h"

namespace kdfm {
namespace wimg {

enum { JOB_FFN = 0, JOB_LNPROJ = 1, JOB_ROWGEMM = 2 };
enum { LP_QKV = 0, LP_GLU = 1 };

// FFN chunk image (csrc/ffn.hip): chunk c, fragment f of CS = 4 DT + 2 KS1 ->
//   W2c(mt, ks2) = 2 mt + ks2 | W1c(ks) = 2 DT + ks | W2Tc(ks) = 2 DT + KS1 + ks | W1Tc(mt, ks2) = 2 DT + 2 KS1 + 2 mt + ks2
__device__ __forceinline__ void ffn_frag(const float* __restrict__ W1, const float* __restrict__ W2, int d, int ff,
                                         int KS1, int DT, int64_t c, int f, int lane, float (&v)[8]) {
  const int r = lane & 31, h = lane >> 5;
  if (f < 2 * DT) {                       // W2[mt*32 + r][c*32 + ks2*16 + 8h + j]
    const int row = (f >> 1) * 32 + r;
    const int64_t col = c * 32 + (f & 1) * 16 + 8 * h;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = row < d ? W2[(int64_t)row * ff + col + j] : 0.f;
  } else if (f < 2 * DT + KS1) {          // W1[c*32 + r][ks*16 + 8h + j]
    const int k0 = (f - 2 * DT) * 16 + 8 * h;
    const int64_t row = c * 32 + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = k0 + j < d ? W1[row * d + k0 + j] : 0.f;
  } else if (f < 2 * DT + 2 * KS1) {      // W2[ks*16 + 8h + j][c*32 + r]
    const int k0 = (f - 2 * DT - KS1) * 16 + 8 * h;
    const int64_t col = c * 32 + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = k0 + j < d ? W2[(int64_t)(k0 + j) * ff + col] : 0.f;
  } else {                                // W1[c*32 + ks2*16 + 8h + j][mt*32 + r]
    const int t = f - 2 * DT - 2 * KS1;
    const int row = (t >> 1) * 32 + r;
    const int64_t k0 = c * 32 + (t & 1) * 16 + 8 * h;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = row < d ? W1[(k0 + j) * d + row] : 0.f;
  }
}

// LN-projection image (csrc/lnproj.hip), fragment f of the forward (bwd = 0) or backward image
__device__ __forceinline__ void lnproj_frag(const float* __restrict__ W, int d, int KS1, int DT, int mode, int bwd,
                                            int f, int lane, float (&v)[8]) {
  const int r = lane & 31, h = lane >> 5;
  const int G = mode == LP_QKV ? 3 : 2;
  int wrow = -1, k0 = 0;
  bool trans = false;
  auto fwd_frag = [&](int g, int t, int ks) {
    const int feat = 32 * t + r;
    wrow = feat < d ? g * d + feat : -1;
    k0 = 16 * ks + 8 * h;
  };
  if (!bwd) {
    if (mode == LP_QKV) {
      const int u = f / KS1, ks = f % KS1;
      fwd_frag(u % 3, u / 3, ks);
    } else {
      const int u = f / (2 * KS1), rem = f % (2 * KS1);
      fwd_frag(rem / KS1, u, rem % KS1);
    }
  } else {
    const int BB = (mode == LP_GLU ? 2 * KS1 : 0) + 2 * G * DT;
    const int t = f / BB;
    int rem = f % BB;
    if (mode == LP_GLU && rem < 2 * KS1) {
      fwd_frag(rem / KS1, t, rem % KS1);
    } else {
      if (mode == LP_GLU) rem -= 2 * KS1;
      const int g = rem / (2 * DT), s2 = (rem / DT) % 2, mt = rem % DT;
      trans = true;
      const int feat0 = 32 * t + 16 * s2 + 8 * h;
      wrow = feat0 < d ? g * d + feat0 : -1;
      k0 = 32 * mt + r;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (wrow < 0) {
      v[j] = 0.f;
    } else if (!trans) {
      v[j] = k0 + j < d ? W[(int64_t)wrow * d + k0 + j] : 0.f;
    } else {
      v[j] = k0 < d ? W[(int64_t)(wrow + j) * d + k0] : 0.f;
    }
  }
}

// row-streaming d x d image (csrc/rowgemm.hip): fragment (mt, ks) of W (trans: W^T)
__device__ __forceinline__ void rowgemm_frag(const float* __restrict__ W, int d, int KS1, int trans, int f, int lane,
                                             float (&v)[8]) {
  const int mt = f / KS1, ks = f % KS1;
  const int o = 32 * mt + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool in = o < d && k0 + j < d;
    v[j] = in ? (trans ? W[(int64_t)(k0 + j) * d + o] : W[(int64_t)o * d + k0 + j]) : 0.f;
  }
}

}  // namespace wimg
}  // namespace kdfm
