// Row-streaming d x d products of a Conformer layer with fused prologues / epilogues (bf16 MFMA, f32
// state; building blocks in lnblock.h): every product whose input AND output are d-wide rows.
//
// Reference: ConformerLayer.forward (built conformer_encoder.py:450-472,
// called :685-692) and its backward:
//   attention linear_out:   x2 = x1 + drop(o W_out^T + b)                    (PRO_NONE, EPI_RESID)
//   conv pointwise_conv2:   x3 = x2 + drop(silu(BN(y)) W_pw2^T + b)           (PRO_BNSILU, EPI_RESID)
//   their data gradients:   do = (drop'(dx2)) W_out,  dz = (drop'(dx3)) W_pw2 (PRO_DROP, EPI_NONE)
// The unfused path ran each as a 64x64-tile GEMM (two column tiles re-reading the rows) plus a
// separate BN-SiLU / dropout pass; here one wave streams 32 rows: the prologue is applied while the
// row is converted to the bf16 B operands (and, for training, stored as the bf16 weight-gradient
// operand: exactly the values the GEMM path rounds at MFMA staging), the d/32 output tiles are
// produced from an LDS-staged weight image, and the epilogue writes f32 rows.
#include "lnblock.h"
#include "wimg.h"

namespace kdfm {
namespace {

using namespace lnb;

constexpr int RG_NT = 128;      // 2 waves = 64 rows per workgroup
constexpr int RG_ROWS = 64;
enum { PRO_NONE = 0, PRO_DROP = 1, PRO_BNSILU = 2 };
enum { EPI_NONE = 0, EPI_RESID = 1 };

// image: fragment (mt, ks), lane (r, h), j: Wop[32 mt + r][16 ks + 8 h + j] with Wop = W (forward,
// W (d, d) as [out][in]) or W^T (data gradient: Wop[o][i] = W[i][o])
__global__ __launch_bounds__(256) void rowgemm_wprep_kernel(const float* __restrict__ W, uint16_t* __restrict__ img,
                                                            int d, int KS1, int trans, int64_t total) {
  const int64_t gidx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gidx >= total) return;
  const int lane = (int)(gidx & 63);
  const int f = (int)(gidx >> 6);
  float v[8];
  wimg::rowgemm_frag(W, d, KS1, trans, f, lane, v);
  *reinterpret_cast<bf16x8*>(img + ((int64_t)f * 64 + lane) * 8) = pack_bf16x8<bf16x8>(v);
}

struct RgArgs {
  const float* x; const uint16_t* img; float* out; int64_t rows; int d;
  // prologue
  float p_in, s_in; const uint64_t* seed; uint64_t st_in;           // PRO_DROP: x * s_in * keep / (1 - p)
  const float* bn_mean; const float* bn_rstd; const float* bn_g; const float* bn_b;   // PRO_BNSILU
  uint16_t* x_h;                                                     // bf16 copy of the prologue output
  // epilogue
  const float* bias; const float* R; float rscale, p_out; uint64_t st_out;
};

template <int KS1, int DT, int PRO, int EPI>
__global__ __launch_bounds__(RG_NT) void rowgemm_kernel(RgArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 img_s[DT * KS1 * FRAG_U4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int64_t row = (int64_t)blockIdx.x * RG_ROWS + wave * 32 + (lane & 31);
  const bool ok = row < a.rows;
  const int d = a.d;
  // weight image -> LDS (all loads first)
  constexpr int UNITS = DT * KS1 * FRAG_U4, PER = (UNITS + RG_NT - 1) / RG_NT;
  const uint4* img = reinterpret_cast<const uint4*>(a.img);
  uint4 pre[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int u = threadIdx.x + RG_NT * i;
    pre[i] = u < UNITS ? img[u] : make_uint4(0, 0, 0, 0);
  }
  const uint64_t seed = (a.p_in > 0.f || a.p_out > 0.f) ? load_seed(a.seed) : 0ull;
  const uint64_t kin = rng_key(seed, a.st_in), kout = rng_key(seed, a.st_out);
  // prologue -> B operands
  bf16x8 bx[KS1];
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const int k0 = ks * 16 + 8 * h;
    const bool in = ok && k0 < d;
    const float4* p = reinterpret_cast<const float4*>(a.x + (in ? row * d + k0 : 0));
    const float4 u = p[0], w = p[1];
    float v[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
    if constexpr (PRO == PRO_DROP) {
      const float ks_in = a.s_in / (1.f - a.p_in);
      bool kp[8] = {true, true, true, true, true, true, true, true};
      if (a.p_in > 0.f)
#pragma unroll
        for (int j = 0; j < 8; j += 2) dropout_keep2_k(kin, (uint64_t)row * d + k0 + j, a.p_in, kp[j], kp[j + 1]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = v[j] * (a.p_in > 0.f ? ks_in : a.s_in);
        if (a.p_in > 0.f) t = kp[j] ? t : 0.f;
        v[j] = t;
      }
    } else if constexpr (PRO == PRO_BNSILU) {
      const int kk = k0 < d ? k0 : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sc = a.bn_rstd[kk + j] * a.bn_g[kk + j];
        v[j] = siluf_((v[j] - a.bn_mean[kk + j]) * sc + a.bn_b[kk + j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = in ? v[j] : 0.f;
    bx[ks] = pack_bf16x8<bf16x8>(v);
    if (a.x_h && in) *reinterpret_cast<bf16x8*>(a.x_h + row * d + k0) = bx[ks];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int u = threadIdx.x + RG_NT * i;
    if (u < UNITS) img_s[u] = pre[i];
  }
  __syncthreads();
  // no early exit for rows past the end: every lane supplies A-operand rows of the MFMAs below
#pragma unroll
  for (int mt = 0; mt < DT; ++mt) {
    f32x16 acc = zero16();
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) acc = mfma32(img_s[(mt * KS1 + ks) * FRAG_U4 + lane], bx[ks], acc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = 32 * mt + 8 * q + 4 * h;
      if (!ok || n0 >= d) continue;
      float o[4] = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
      if constexpr (EPI == EPI_RESID) {
        const float4 bb = a.bias ? *reinterpret_cast<const float4*>(a.bias + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 rr = *reinterpret_cast<const float4*>(a.R + row * d + n0);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w}, rv[4] = {rr.x, rr.y, rr.z, rr.w};
        const float ks_out = 1.f / (1.f - a.p_out);
        bool kp[4] = {true, true, true, true};
        if (a.p_out > 0.f) {
          dropout_keep2_k(kout, (uint64_t)row * d + n0, a.p_out, kp[0], kp[1]);
          dropout_keep2_k(kout, (uint64_t)row * d + n0 + 2, a.p_out, kp[2], kp[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = o[i] + bv[i];
          if (a.p_out > 0.f) v = kp[i] ? v * ks_out : 0.f;
          o[i] = rv[i] + a.rscale * v;
        }
      }
      *reinterpret_cast<float4*>(a.out + row * d + n0) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

template <int KS1, int DT>
int rg_launch(int pro, int epi, const RgArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)ceil_div(a.rows, RG_ROWS)), blk(RG_NT);
#define RG_CASE(P, E)                                                                \
  if (pro == P && epi == E) {                                                        \
    hipLaunchKernelGGL((rowgemm_kernel<KS1, DT, P, E>), grid, blk, 0, st, a);        \
    return check_launch("kdfm_rowgemm");                                             \
  }
  RG_CASE(PRO_NONE, EPI_RESID)
  RG_CASE(PRO_BNSILU, EPI_RESID)
  RG_CASE(PRO_DROP, EPI_NONE)
  RG_CASE(PRO_NONE, EPI_NONE)
#undef RG_CASE
  set_error("kdfm_rowgemm: unsupported prologue / epilogue combination");
  return KDFM_EUNSUPPORTED;
}

}  // namespace
}  // namespace kdfm

extern "C" {

int64_t kdfm_rowgemm_img_elems(int64_t d) {
  int KS1, DT;
  if (kdfm::lnb::ln_dims(d, KS1, DT) != 0) return 0;
  return (int64_t)DT * KS1 * 512;
}

int kdfm_rowgemm_wprep(const float* W, uint16_t* img, int64_t d, int32_t trans, void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(W && img, "null pointer");
  int KS1, DT;
  KDFM_REQUIRE(ln_dims(d, KS1, DT) == 0, "unsupported d");
  KDFM_REQUIRE(al16(img), "img must be 16-byte aligned");
  const int64_t total = (int64_t)DT * KS1 * 64;
  hipLaunchKernelGGL(rowgemm_wprep_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, as_stream(stream), W,
                     img, (int)d, KS1, (int)trans, total);
  return check_launch("kdfm_rowgemm_wprep");
}

int kdfm_rowgemm(const float* x, const uint16_t* img, float* out, int64_t rows, int64_t d, int32_t prologue,
                 float p_in, float s_in, uint64_t stream_in, const float* bn_mean, const float* bn_rstd,
                 const float* bn_g, const float* bn_b, uint16_t* x_h, int32_t epilogue, const float* bias,
                 const float* R, float rscale, float p_out, uint64_t stream_out, const uint64_t* seed,
                 void* stream) {
  using namespace kdfm;
  using namespace kdfm::lnb;
  KDFM_REQUIRE(x && img && out, "null pointer");
  int KS1, DT;
  KDFM_REQUIRE(ln_dims(d, KS1, DT) == 0, "unsupported d");
  KDFM_REQUIRE(al16(x) && al16(img) && al16(out) && al16(x_h) && al16(bias) && al16(R), "operands must be 16-byte aligned");
  KDFM_REQUIRE(prologue != PRO_BNSILU || (bn_mean && bn_rstd && bn_g && bn_b), "BN-SiLU prologue needs its statistics");
  KDFM_REQUIRE(epilogue != EPI_RESID || R, "residual epilogue needs R");
  KDFM_REQUIRE(p_in >= 0.f && p_in < 1.f && p_out >= 0.f && p_out < 1.f, "dropout p");
  KDFM_REQUIRE((p_in == 0.f && p_out == 0.f) || seed, "dropout needs a seed");
  if (rows <= 0) return KDFM_OK;
  RgArgs a{x, img, out, rows, (int)d, p_in, s_in, seed, stream_in, bn_mean, bn_rstd, bn_g, bn_b, x_h,
           bias, R, rscale, p_out, stream_out};
  hipStream_t st = as_stream(stream);
  if (KS1 == 6) return rg_launch<6, 3>(prologue, epilogue, a, st);
  if (KS1 == 11) return rg_launch<11, 6>(prologue, epilogue, a, st);
  return rg_launch<12, 6>(prologue, epilogue, a, st);
}

}  // extern "C"
