// Log-mel frontend (NeMo AudioToMelSpectrogramPreprocessor -> FilterbankFeatures, called at
// audio_preprocessing.py:299-300; semantics SURVEY.md Appendix A.1) and SpecAugment (A.2),
// plus the im2col/col2im of the striding ConvSubsampling (A.3, built conformer_encoder.py:381-390).
//
// STFT-as-GEMM: the frames of the zero-centre-padded, pre-emphasised signal are read as a strided
// view (frame t = samples [160t+56, 160t+456) of the padded row) and multiplied by a 400 x 514
// basis (Hann(400) folded into cos / -sin) in the MFMA GEMM; this file holds the surrounding
// memory-bound passes.
#include "common.h"

namespace kdfm {
namespace {

// xp[b, pad + n] = preemph(x + dither*noise)[n] masked to n < len;  zero halo of `pad` each side
__global__ __launch_bounds__(256) void preemph_pad_kernel(const float* __restrict__ x, const int64_t* __restrict__ lens,
                                                          float* __restrict__ xp, int64_t N, int64_t pad, float coef,
                                                          float dither, const uint64_t* seed_ptr, uint64_t rng_stream) {
  const int64_t b = blockIdx.y;
  const int64_t W = N + 2 * pad;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= W) return;
  const int64_t n = j - pad;
  float v = 0.f;
  const int64_t len = lens ? lens[b] : N;
  if (n >= 0 && n < N && n < len) {
    const float* xr = x + b * N;
    float cur = xr[n];
    if (dither > 0.f) cur += dither * rng_normal(load_seed(seed_ptr), rng_stream, (uint64_t)(b * N + n));
    if (n == 0) {
      v = cur;
    } else {
      float prev = xr[n - 1];
      if (dither > 0.f) prev += dither * rng_normal(load_seed(seed_ptr), rng_stream, (uint64_t)(b * N + n - 1));
      v = cur - coef * prev;
    }
  }
  xp[b * W + j] = v;
}

// pw[r, f] = spec[r, f]^2 + spec[r, F + f]^2   (spec rows = [re(0..F-1) | im(0..F-1)])
__global__ __launch_bounds__(256) void power_kernel(const float* __restrict__ spec, float* __restrict__ pw, int64_t rows,
                                                    int64_t F) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * F) return;
  const int64_t r = idx / F, f = idx - r * F;
  const float re = spec[r * 2 * F + f], im = spec[r * 2 * F + F + f];
  pw[idx] = re * re + im * im;
}

// out[b,t,j] = (log(mel+guard) - mean_j) / (std_j + 1e-5) for t < seq_len, 0 beyond
// mean/std over valid frames, unbiased (n-1) std; block = (b, 64 mel columns), 4 frame lanes.
__global__ __launch_bounds__(256) void logmel_norm_kernel(const float* __restrict__ mel, const int64_t* __restrict__ sl,
                                                          float* __restrict__ out, int64_t T, int64_t nf, float guard) {
  __shared__ float red[4][64];
  const int64_t b = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  const int64_t n = sl[b] < T ? sl[b] : T;
  const float* mr = mel + b * T * nf;
  float* orow = out + b * T * nf;
  float s = 0.f;
  if (j < nf)
    for (int64_t t = w; t < n; t += 4) s += __logf(mr[t * nf + j] + guard);
  red[w][lane] = s;
  __syncthreads();
  const float mean = (red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]) / (float)n;
  __syncthreads();
  float q = 0.f;
  if (j < nf)
    for (int64_t t = w; t < n; t += 4) {
      const float dv = __logf(mr[t * nf + j] + guard) - mean;
      q += dv * dv;
    }
  red[w][lane] = q;
  __syncthreads();
  float var = (red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]) / ((float)n - 1.f);
  float sd = sqrtf(var);
  if (!(sd == sd)) sd = 0.f;  // n == 1 -> nan -> 0 (normalize_batch edge case)
  const float inv = 1.f / (sd + 1e-5f);
  if (j < nf)
    for (int64_t t = w; t < T; t += 4) orow[t * nf + j] = (t < n) ? (__logf(mr[t * nf + j] + guard) - mean) * inv : 0.f;
}

// Register-resident form for T <= 32 * LM_PER frames: block = (b, 8 mel columns), 256 threads =
// 8 columns x 32 frame lanes; every log value of the block's slice is loaded once (all loads in
// flight together) and kept in registers across the mean, the variance and the write pass.
constexpr int LM_PER = 64;
__global__ __launch_bounds__(256) void logmel_norm_reg_kernel(const float* __restrict__ mel, const int64_t* __restrict__ sl,
                                                              float* __restrict__ out, int T, int nf, float guard) {
  __shared__ float red[32][9];
  const int b = blockIdx.y;
  const int fl = threadIdx.x & 7, tg = threadIdx.x >> 3;
  const int j = blockIdx.x * 8 + fl;
  const int n = (int)(sl[b] < T ? sl[b] : T);
  const float* mr = mel + (int64_t)b * T * nf;
  float* orow = out + (int64_t)b * T * nf;
  float l[LM_PER];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LM_PER; ++k) {
    const int t = tg + 32 * k;
    l[k] = (j < nf && t < n) ? __logf(mr[(int64_t)t * nf + j] + guard) : 0.f;
    s += l[k];
  }
  red[tg][fl] = s;
  __syncthreads();
  float tot = 0.f;
#pragma unroll 8
  for (int q = 0; q < 32; ++q) tot += red[q][fl];
  const float mean = tot / (float)n;
  __syncthreads();
  float qv = 0.f;
#pragma unroll
  for (int k = 0; k < LM_PER; ++k) {
    const int t = tg + 32 * k;
    const float dv = (t < n) ? l[k] - mean : 0.f;
    qv += dv * dv;
  }
  red[tg][fl] = qv;
  __syncthreads();
  float var = 0.f;
#pragma unroll 8
  for (int q = 0; q < 32; ++q) var += red[q][fl];
  var /= ((float)n - 1.f);
  float sd = sqrtf(var);
  if (!(sd == sd)) sd = 0.f;
  const float inv = 1.f / (sd + 1e-5f);
  if (j < nf) {
#pragma unroll
    for (int k = 0; k < LM_PER; ++k) {
      const int t = tg + 32 * k;
      if (t < T) orow[(int64_t)t * nf + j] = (t < n) ? (l[k] - mean) * inv : 0.f;
    }
  }
}

// SpecAugment, NeMo's vectorized form (SpectrogramAugmentation(use_vectorized_spec_augment=True), the
// default at audio_preprocessing.py:490-520), per utterance b and mask q with
// uniforms U in [0, 1) (f32 arithmetic, truncation toward zero as torch's .long()):
//   time:  w = (int)(U_w * min(time_width * len, T)),  start = (int)(U_s * (float)(len - w))
//   freq:  w = (int)(U_w * freq_width),                start = (int)(U_s * (float)(nf - w))
// cells with start <= index < start + w are set to 0.  The uniforms come from `uni` when given (parity
// mode, SURVEY.md §8(b): RNG as an input) laid out uni[b][4 q'] for [time widths (tmasks) | time starts
// (tmasks) | freq widths (fmasks) | freq starts (fmasks)], else from the counter RNG (time mask q: indices
// b*64 + 32 + 2q, + 1; frequency mask q: b*64 + 2q, + 1).
// One block per (utterance, chunk of SA_EPB cells): the utterance's mask intervals are computed once into
// LDS by the first fmasks + tmasks threads, then every cell tests against them.
constexpr int SA_EPB = 256 * 8;
__global__ __launch_bounds__(256) void specaug_kernel(float* __restrict__ x, const int64_t* __restrict__ sl,
                                                      uint8_t* __restrict__ mask_out, int64_t B, int64_t T, int64_t nf,
                                                      int fmasks, int fwidth, int tmasks, float twidth,
                                                      const uint64_t* seed_ptr, uint64_t st,
                                                      const float* __restrict__ uni) {
  __shared__ int lo[32], hi[32];   // [0, fmasks): frequency bands; [fmasks, fmasks + tmasks): time bands
  const int64_t b = blockIdx.y;
  const int64_t cells = T * nf;
  const int64_t len = sl[b];
  if (threadIdx.x < fmasks + tmasks) {
    const int q = threadIdx.x;
    const float* ub = uni ? uni + b * 2 * (fmasks + tmasks) : nullptr;
    float uw, us;
    if (q < fmasks) {
      if (ub) {
        uw = ub[2 * tmasks + q];
        us = ub[2 * tmasks + fmasks + q];
      } else {
        const uint64_t seed = load_seed(seed_ptr);
        const uint64_t base = (uint64_t)b * 64 + (uint64_t)q * 2;
        uw = rng_uniform(seed, st, base);
        us = rng_uniform(seed, st, base + 1);
      }
      const int64_t w = (int64_t)(uw * (float)fwidth);
      const int64_t s0 = (int64_t)(us * (float)(nf - w));
      lo[q] = (int)s0;
      hi[q] = (int)(s0 + w);
    } else {
      const int qt = q - fmasks;
      if (ub) {
        uw = ub[qt];
        us = ub[tmasks + qt];
      } else {
        const uint64_t seed = load_seed(seed_ptr);
        const uint64_t base = (uint64_t)b * 64 + 32 + (uint64_t)qt * 2;
        uw = rng_uniform(seed, st, base);
        us = rng_uniform(seed, st, base + 1);
      }
      const float wmax = fminf(twidth * (float)len, (float)T);
      const int64_t w = (int64_t)(uw * wmax);
      const int64_t s0 = (int64_t)(us * (float)(len - w));
      lo[q] = (int)s0;
      hi[q] = (int)(s0 + w);
    }
  }
  __syncthreads();
  const int n = (int)nf;
  for (int64_t c = (int64_t)blockIdx.x * SA_EPB + threadIdx.x; c < min<int64_t>(cells, (int64_t)(blockIdx.x + 1) * SA_EPB);
       c += 256) {
    const int t = (int)(c / n), f = (int)(c - (int64_t)t * n);
    bool m = false;
    for (int q = 0; q < fmasks; ++q) m |= f >= lo[q] && f < hi[q];
    for (int q = fmasks; q < fmasks + tmasks; ++q) m |= t >= lo[q] && t < hi[q];
    const int64_t idx = b * cells + c;
    if (m) x[idx] = 0.f;
    if (mask_out) mask_out[idx] = m ? 1 : 0;
  }
}

// cols[(b,t2,f2), c*9 + ky*3 + kx] = X[b, 2*t2-1+ky, 2*f2-1+kx, c]  (0 outside / beyond len_in)
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ X, const int64_t* __restrict__ lin,
                                                     float* __restrict__ cols, int64_t B, int64_t T1, int64_t F1,
                                                     int64_t C, int64_t T2, int64_t F2) {
  const int64_t idx = xcd_block() * 256 + threadIdx.x;
  const int64_t KC = 9 * C;
  if (idx >= B * T2 * F2 * KC) return;
  const int64_t q = idx % KC, row = idx / KC;
  const int64_t c = q / 9, tap = q % 9, ky = tap / 3, kx = tap % 3;
  const int64_t f2 = row % F2, t2 = (row / F2) % T2, b = row / (F2 * T2);
  const int64_t t1 = 2 * t2 - 1 + ky, f1 = 2 * f2 - 1 + kx;
  float v = 0.f;
  const int64_t len = lin ? lin[b] : T1;
  if (t1 >= 0 && t1 < T1 && t1 < len && f1 >= 0 && f1 < F1) v = X[((b * T1 + t1) * F1 + f1) * C + c];
  cols[idx] = v;
}


// ---- STFT power + mel filterbank via a 512-point real FFT per frame ------------------------------
// FilterbankFeatures (audio_preprocessing.py:93-103, 214-300): |STFT|^2 of the Hann(400)-windowed
// frame centred in n_fft = 512, then the Slaney mel filterbank.  The DFT-as-GEMM formulation costs
// 2 x 512 x 514 flops per frame on f32 MFMA; here one wave owns a frame and runs the real FFT as a
// 256-point complex radix-2 decimation-in-frequency FFT of z[m] = s[2m] + i s[2m+1] IN REGISTERS:
// lane l holds z[l + 64 q], q = 0..3, so the spans 128 and 64 pair a lane's own registers and the
// spans 32..1 pair lane l with lane l ^ span, exchanged by DPP row permutations (1, 2, 4, 8) and
// v_permlane16/32_swap (16, 32) -- no LDS traffic until the bit-reversed result is stored once
// (the radix-2 stages in LDS cost 8 read+write passes per frame and bound the kernel on the LDS
// pipe); twiddles e^{-2 pi i j / 512} from a host-computed table, held per lane in registers.
// Then the real-FFT split
//   X[k] = (Z[k] + conj Z[256-k]) / 2 - i W^k (Z[k] - conj Z[256-k]) / 2,   W = e^{-2 pi i / 512},
// |X[k]|^2 for k = 0..256, and each mel filter's dot product over its nonzero bin range
// [fb_lo, fb_hi).  Output mel (B*T, nfilt) f32 (log + per-feature normalisation follow).
constexpr int FFT_N = 512, FFT_H = 256, FFT_WAVES = 16;

// wave-local LDS hand-off (each wave owns its buffers): drain this wave's LDS ops; the asm's memory
// clobber keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void fft_wsync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int bitrev8(int v) { return (int)(__builtin_bitreverse32((uint32_t)v) >> 24); }

// v from lane (lane ^ D) of the wave: DPP quad / row permutations for D <= 8 (xor 4 = xor 3 then xor 7,
// xor 8 = xor 7 then xor 15), the gfx950 half-row / half-wave swaps for 16 and 32 (swap(x, x) returns
// [own lower part in both | own upper part in both]: the partner's value is the other one)
template <int D>
__device__ __forceinline__ float lane_xor(float v, int lane) {
  const int i = __builtin_bit_cast(int, v);
  int r;
  if constexpr (D == 1) {
    r = __builtin_amdgcn_mov_dpp(i, 0xB1, 0xF, 0xF, false);                 // quad_perm [1,0,3,2]
  } else if constexpr (D == 2) {
    r = __builtin_amdgcn_mov_dpp(i, 0x4E, 0xF, 0xF, false);                 // quad_perm [2,3,0,1]
  } else if constexpr (D == 4) {
    r = __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(i, 0x1B, 0xF, 0xF, false), 0x141, 0xF, 0xF, false);
  } else if constexpr (D == 8) {
    r = __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(i, 0x141, 0xF, 0xF, false), 0x140, 0xF, 0xF, false);
  } else if constexpr (D == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(i, i, false, false);
    r = (lane & 16) ? (int)p[0] : (int)p[1];
  } else {
    static_assert(D == 32, "span");
    const auto p = __builtin_amdgcn_permlane32_swap(i, i, false, false);
    r = (lane & 32) ? (int)p[0] : (int)p[1];
  }
  return __builtin_bit_cast(float, r);
}

__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}

// DIF stage of span D < 64 across lanes: the lane without bit D keeps a + b, the lane with it takes
// (a - b) w (w = 1 on the lower lanes, so the twiddle multiply is branch-free)
template <int D>
__device__ __forceinline__ void dif_lanes(float2 (&z)[4], int lane, float2 w) {
  const float sg = (lane & D) ? -1.f : 1.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float yx = lane_xor<D>(z[q].x, lane), yy = lane_xor<D>(z[q].y, lane);
    const float2 u = make_float2(fmaf(sg, z[q].x, yx), fmaf(sg, z[q].y, yy));
    z[q] = D == 1 ? u : cmul(u, w);
  }
}

constexpr int FB_LDS = 4096;   // compact filterbank (nonzero ranges of every filter) staged per workgroup

__global__ __launch_bounds__(64 * FFT_WAVES) void logmel_fft_kernel(
    const float* __restrict__ xp, int64_t ldx, const float* __restrict__ win, const float2* __restrict__ tw,
    const float* __restrict__ fb, const int* __restrict__ fb_lo, const int* __restrict__ fb_hi, float* __restrict__ mel,
    int64_t B, int64_t T, int hop, int off, int nwin, int nfilt, int nbins) {
  __shared__ float2 Zs[FFT_WAVES][FFT_H];
  __shared__ float Pw[FFT_WAVES][FFT_H + 8];
  __shared__ float2 W[FFT_N];
  __shared__ float Fc[FB_LDS];          // filter m's weights for bins [lo_m, hi_m) at Fc[Fo[m] ...]
  __shared__ int Fo[256 + 1], Flo[256], Fn[256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < FFT_N; e += 64 * FFT_WAVES) W[e] = tw[e];
  // the mel filterbank is ~2 nonzero weights per bin (triangular filters): its nonzero ranges go to LDS
  // once per workgroup, so the per-frame dot products read LDS instead of waiting on global loads
  for (int m = threadIdx.x; m < nfilt; m += 64 * FFT_WAVES) {
    const int lo = fb_lo[m], hi = fb_hi[m];
    Flo[m] = lo;
    Fn[m] = hi > lo ? hi - lo : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int o = 0;
    for (int m = 0; m < nfilt; ++m) {
      Fo[m] = o;
      o += Fn[m];
    }
    Fo[nfilt] = o;
  }
  __syncthreads();
  const int total = Fo[nfilt];
  const bool staged = total <= FB_LDS;
  if (staged) {   // flat over the nonzero weights: every thread's loads are independent and in flight together
    constexpr int PER = FB_LDS / (64 * FFT_WAVES);
    float v[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int e = threadIdx.x + it * 64 * FFT_WAVES;
      v[it] = 0.f;
      if (e < total) {
        int lo = 0, hi = nfilt - 1;   // the filter m with Fo[m] <= e < Fo[m + 1]
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (Fo[mid] <= e) lo = mid; else hi = mid - 1;
        }
        v[it] = fb[(int64_t)lo * nbins + Flo[lo] + (e - Fo[lo])];
      }
    }
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int e = threadIdx.x + it * 64 * FFT_WAVES;
      if (e < total) Fc[e] = v[it];
    }
  }
  __syncthreads();
  float2* Z = Zs[w];
  float* P = Pw[w];
  const int64_t nframes = B * T;
  // the window taps of this lane's 8 samples are the same for every frame: registers, loaded once
  float wv[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n0 = 2 * (lane + 64 * q), n1 = n0 + 1;
    wv[2 * q] = (n0 >= off && n0 < off + nwin) ? win[n0 - off] : 0.f;
    wv[2 * q + 1] = (n1 >= off && n1 < off + nwin) ? win[n1 - off] : 0.f;
  }
  // per-lane DIF twiddles W_{2D}^{e mod D} = W512^{(e mod D) 256 / D} of every span D (the lower lanes
  // of a cross-lane span multiply by 1)
  float2 t128[2], t64, tl[5];
  t128[0] = W[2 * lane];
  t128[1] = W[2 * lane + 128];
  t64 = W[4 * lane];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int D = 32 >> s;
    tl[s] = (lane & D) ? W[(lane & (D - 1)) * (256 / D)] : make_float2(1.f, 0.f);
  }
  // software pipeline: the next frame's samples are loaded while this frame is transformed
  const int64_t fstep = (int64_t)gridDim.x * FFT_WAVES;
  float2 nx[4];
  auto fetch = [&](int64_t fr) {
    const int64_t b = fr / T, t = fr - b * T;
    const float* src = xp + b * ldx + t * hop;
#pragma unroll
    for (int q = 0; q < 4; ++q) nx[q] = *reinterpret_cast<const float2*>(src + 2 * (lane + 64 * q));
  };
  int64_t f = (int64_t)blockIdx.x * FFT_WAVES + w;
  if (f < nframes) fetch(f);
  for (; f < nframes; f += fstep) {
    // z[m] = s[2m] + i s[2m+1], s[n] = win[n - off] x[t hop + n] on [off, off + nwin); lane holds m = lane + 64 q
    float2 z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) z[q] = make_float2(wv[2 * q] * nx[q].x, wv[2 * q + 1] * nx[q].y);
    if (f + fstep < nframes) fetch(f + fstep);
    // spans 128 and 64: within the lane's registers
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float2 a = z[q], b = z[q + 2];
      z[q] = make_float2(a.x + b.x, a.y + b.y);
      z[q + 2] = cmul(make_float2(a.x - b.x, a.y - b.y), t128[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      const float2 a = z[q], b = z[q + 1];
      z[q] = make_float2(a.x + b.x, a.y + b.y);
      z[q + 1] = cmul(make_float2(a.x - b.x, a.y - b.y), t64);
    }
    dif_lanes<32>(z, lane, tl[0]);
    dif_lanes<16>(z, lane, tl[1]);
    dif_lanes<8>(z, lane, tl[2]);
    dif_lanes<4>(z, lane, tl[3]);
    dif_lanes<2>(z, lane, tl[4]);
    dif_lanes<1>(z, lane, make_float2(1.f, 0.f));
    // element e = lane + 64 q now holds Z[bitrev8(e)]
#pragma unroll
    for (int q = 0; q < 4; ++q) Z[bitrev8(lane + 64 * q)] = z[q];
    fft_wsync();   // this wave's LDS writes complete before its reads
    // real-FFT split and power
    for (int k = lane; k < nbins; k += 64) {
      const float2 zk = Z[k & (FFT_H - 1)], zr = Z[(FFT_H - k) & (FFT_H - 1)];
      const float er = 0.5f * (zk.x + zr.x), ei = 0.5f * (zk.y - zr.y);          // (Zk + conj Zr) / 2
      const float dr = 0.5f * (zk.x - zr.x), di = 0.5f * (zk.y + zr.y);          // (Zk - conj Zr) / 2
      const float2 wk = W[k & (FFT_N - 1)];
      // -i W^k (dr + i di) = (wk.y dr + wk.x di) + i (wk.y di - wk.x dr)
      const float xr = er + (wk.x * di + wk.y * dr);
      const float xi = ei + (wk.y * di - wk.x * dr);
      P[k] = xr * xr + xi * xi;
    }
    fft_wsync();
    float* out = mel + f * nfilt;
    for (int m = lane; m < nfilt; m += 64) {
      const int lo = Flo[m], nk = Fn[m];
      float acc = 0.f;
      if (staged) {   // four independent partial sums: the LDS reads of a filter's bins overlap
        const float* fr = Fc + Fo[m];
        const float* pp = P + lo;
        float a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int k = 0;
        for (; k + 4 <= nk; k += 4) {
          acc = fmaf(fr[k], pp[k], acc);
          a1 = fmaf(fr[k + 1], pp[k + 1], a1);
          a2 = fmaf(fr[k + 2], pp[k + 2], a2);
          a3 = fmaf(fr[k + 3], pp[k + 3], a3);
        }
        for (; k < nk; ++k) acc = fmaf(fr[k], pp[k], acc);
        acc = (acc + a1) + (a2 + a3);
      } else {
        const float* row = fb + (int64_t)m * nbins + lo;
        for (int k = 0; k < nk; ++k) acc = fmaf(row[k], P[lo + k], acc);
      }
      out[m] = acc;
    }
    fft_wsync();   // Z / P are rewritten by the next frame
  }
}

// TAP-MAJOR bf16 variant: cols[(b,t2,f2), tap*C + c] = bf16(X[b, 2*t2-1+ky, 2*f2-1+kx, c]); one thread
// per 8 consecutive channels of one (row, tap): two coalesced float4 reads, one 16-byte store.  The
// bf16 column matrix is the weight-gradient operand of the bf16 step (half the bytes of the f32 one).
template <typename TX>
__global__ __launch_bounds__(256) void im2col_tm_bf16_kernel(const TX* __restrict__ X, const int64_t* __restrict__ lin,
                                                             uint16_t* __restrict__ cols, int64_t B, int64_t T1,
                                                             int64_t F1, int C, int64_t T2, int64_t F2) {
  const int64_t idx = xcd_block() * 256 + threadIdx.x;
  const int CG = C >> 3;
  if (idx >= B * T2 * F2 * 9 * CG) return;
  const int cg = (int)(idx % CG);
  const int64_t rt = idx / CG;
  const int tap = (int)(rt % 9);
  const int64_t row = rt / 9;
  const int ky = tap / 3, kx = tap - 3 * (tap / 3);
  const int64_t f2 = row % F2, t2 = (row / F2) % T2, b = row / (F2 * T2);
  const int64_t t1 = 2 * t2 - 1 + ky, f1 = 2 * f2 - 1 + kx;
  const int64_t len = lin ? lin[b] : T1;
  typedef __attribute__((ext_vector_type(8))) short bf8;
  const bool in = t1 >= 0 && t1 < T1 && t1 < len && f1 >= 0 && f1 < F1;
  bf8* dst = reinterpret_cast<bf8*>(cols + row * 9 * C + tap * C + 8 * cg);
  if constexpr (sizeof(TX) == 2) {   // bf16 source: a 16-byte copy
    *dst = in ? *reinterpret_cast<const bf8*>(X + ((b * T1 + t1) * F1 + f1) * C + 8 * cg) : bf8{0, 0, 0, 0, 0, 0, 0, 0};
  } else {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (in) {
      const float* src = X + ((b * T1 + t1) * F1 + f1) * C + 8 * cg;
      const float4 a = *reinterpret_cast<const float4*>(src), c = *reinterpret_cast<const float4*>(src + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    }
    *dst = pack_bf16x8<bf8>(v);
  }
}

// dX[b,t1,f1,c] = sum over taps hitting (t1,f1) of dcols; zero beyond len_in; *= (aux > 0) if aux.
// TAPMAJOR: dcols columns are tap*C + c (the lanes of a wave, consecutive c, read one contiguous run
// per tap) instead of c*9 + tap (stride-9 lanes: 36 partially used lines per load).
template <bool TAPMAJOR>
__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcols, const int64_t* __restrict__ lin,
                                                     const float* __restrict__ aux, float* __restrict__ dX, int64_t B,
                                                     int64_t T1, int64_t F1, int64_t C, int64_t T2, int64_t F2) {
  const int64_t idx = xcd_block() * 256 + threadIdx.x;
  if (idx >= B * T1 * F1 * C) return;
  const int64_t c = idx % C, f1 = (idx / C) % F1, t1 = (idx / (C * F1)) % T1, b = idx / (C * F1 * T1);
  const int64_t len = lin ? lin[b] : T1;
  float acc = 0.f;
  if (t1 < len) {
    for (int ky = 0; ky < 3; ++ky) {
      const int64_t tn = t1 + 1 - ky;
      if (tn < 0 || (tn & 1)) continue;
      const int64_t t2 = tn >> 1;
      if (t2 >= T2) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int64_t fn = f1 + 1 - kx;
        if (fn < 0 || (fn & 1)) continue;
        const int64_t f2 = fn >> 1;
        if (f2 >= F2) continue;
        const int64_t cell = ((b * T2 + t2) * F2 + f2) * 9 * C;
        acc += TAPMAJOR ? dcols[cell + (ky * 3 + kx) * C + c] : dcols[cell + c * 9 + ky * 3 + kx];
      }
    }
    if (aux && !(aux[idx] > 0.f)) acc = 0.f;
  }
  dX[idx] = acc;
}

}  // namespace
}  // namespace kdfm

extern "C" {

int kdfm_preemph_pad(const float* wav, const int64_t* lengths, float* xp, int64_t B, int64_t N, int64_t pad,
                     float preemph, float dither, const uint64_t* seed, uint64_t rng_stream, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(wav && xp, "null pointer");
  KDFM_REQUIRE(B >= 0 && N >= 0 && pad >= 0, "bad shape");
  KDFM_REQUIRE(dither == 0.f || seed, "dither needs a seed");
  if (B == 0) return KDFM_OK;
  dim3 grid((unsigned)ceil_div(N + 2 * pad, 256), (unsigned)B);
  hipLaunchKernelGGL(preemph_pad_kernel, grid, dim3(256), 0, as_stream(stream), wav, lengths, xp, N, pad, preemph,
                     dither, seed, rng_stream);
  return check_launch("kdfm_preemph_pad");
}

int kdfm_logmel_fft(const float* xp, int64_t ldx, const float* window, const float* twiddle, const float* fb,
                    const int32_t* fb_lo, const int32_t* fb_hi, float* mel, int64_t B, int64_t T, int64_t hop,
                    int64_t n_fft, int64_t win, int64_t nfilt, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(xp && window && twiddle && fb && fb_lo && fb_hi && mel, "null pointer");
  KDFM_REQUIRE(n_fft == FFT_N && win > 0 && win <= n_fft && nfilt > 0 && nfilt <= 256 && hop > 0,
               "n_fft must be 512, at most 256 filters");
  if (B * T == 0) return KDFM_OK;
  const int64_t groups = ceil_div(B * T, FFT_WAVES);
  static const int64_t cap = [] {   // workgroups (frames are grid-strided); KDFM_FFT_GRID overrides
    const char* v = getenv("KDFM_FFT_GRID");
    return v && atoi(v) > 0 ? (int64_t)atoi(v) : (int64_t)512;
  }();
  const unsigned grid = (unsigned)(groups < cap ? groups : cap);
  hipLaunchKernelGGL(logmel_fft_kernel, dim3(grid), dim3(64 * FFT_WAVES), 0, as_stream(stream), xp, ldx, window,
                     reinterpret_cast<const float2*>(twiddle), fb, fb_lo, fb_hi, mel, B, T, (int)hop,
                     (int)((n_fft - win) / 2), (int)win, (int)nfilt, (int)(n_fft / 2 + 1));
  return check_launch("kdfm_logmel_fft");
}

int kdfm_power_spectrum(const float* spec, float* power, int64_t rows, int64_t nbins, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(spec && power, "null pointer");
  const int64_t n = rows * nbins;
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(power_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), spec, power,
                     rows, nbins);
  return check_launch("kdfm_power_spectrum");
}

int kdfm_logmel_normalize(const float* mel, const int64_t* seq_len, float* out, int64_t B, int64_t T, int64_t nfilt,
                          float log_guard, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(mel && seq_len && out, "null pointer");
  if (B * T * nfilt == 0) return KDFM_OK;
  if (T <= 32 * LM_PER) {
    dim3 grid((unsigned)ceil_div(nfilt, 8), (unsigned)B);
    hipLaunchKernelGGL(logmel_norm_reg_kernel, grid, dim3(256), 0, as_stream(stream), mel, seq_len, out, (int)T,
                       (int)nfilt, log_guard);
    return check_launch("kdfm_logmel_normalize");
  }
  dim3 grid((unsigned)ceil_div(nfilt, 64), (unsigned)B);
  hipLaunchKernelGGL(logmel_norm_kernel, grid, dim3(256), 0, as_stream(stream), mel, seq_len, out, T, nfilt,
                     log_guard);
  return check_launch("kdfm_logmel_normalize");
}

int kdfm_specaugment(float* x, const int64_t* seq_len, uint8_t* mask_out, int64_t B, int64_t T, int64_t nfilt,
                     int32_t freq_masks, int32_t freq_width, int32_t time_masks, float time_width,
                     const uint64_t* seed, uint64_t rng_stream, const float* uniforms, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && seq_len && (seed || uniforms), "null pointer");
  KDFM_REQUIRE(freq_masks >= 0 && freq_masks <= 16 && time_masks >= 0 && time_masks <= 16, "mask counts in [0,16]");
  const int64_t n = B * T * nfilt;
  if (n == 0) return KDFM_OK;
  KDFM_REQUIRE(freq_masks + time_masks <= 32, "at most 32 masks");
  hipLaunchKernelGGL(specaug_kernel, dim3((unsigned)ceil_div(T * nfilt, SA_EPB), (unsigned)B), dim3(256), 0,
                     as_stream(stream), x, seq_len, mask_out, B, T, nfilt, freq_masks, freq_width, time_masks,
                     time_width, seed, rng_stream, uniforms);
  return check_launch("kdfm_specaugment");
}

int kdfm_im2col_3x3s2(const float* X, const int64_t* len_in, float* cols, int64_t B, int64_t T1, int64_t F1, int64_t C,
                      void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(X && cols, "null pointer");
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  const int64_t n = B * T2 * F2 * 9 * C;
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), X, len_in,
                     cols, B, T1, F1, C, T2, F2);
  return check_launch("kdfm_im2col_3x3s2");
}

int kdfm_im2col_3x3s2_tm_bf16(const float* X, const int64_t* len_in, uint16_t* cols, int64_t B, int64_t T1, int64_t F1,
                              int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(X && cols, "null pointer");
  KDFM_REQUIRE(C % 8 == 0 && ((((uintptr_t)X) | ((uintptr_t)cols)) & 15) == 0, "C % 8 and 16-byte alignment");
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  const int64_t n = B * T2 * F2 * 9 * (C / 8);
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(im2col_tm_bf16_kernel<float>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), X,
                     len_in, cols, B, T1, F1, (int)C, T2, F2);
  return check_launch("kdfm_im2col_3x3s2_tm_bf16");
}

int kdfm_im2col_3x3s2_tm_from_bf16(const uint16_t* X, const int64_t* len_in, uint16_t* cols, int64_t B, int64_t T1,
                                   int64_t F1, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(X && cols, "null pointer");
  KDFM_REQUIRE(C % 8 == 0 && ((((uintptr_t)X) | ((uintptr_t)cols)) & 15) == 0, "C % 8 and 16-byte alignment");
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  const int64_t n = B * T2 * F2 * 9 * (C / 8);
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(im2col_tm_bf16_kernel<uint16_t>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                     as_stream(stream), X, len_in, cols, B, T1, F1, (int)C, T2, F2);
  return check_launch("kdfm_im2col_3x3s2_tm_from_bf16");
}

int kdfm_col2im_3x3s2(const float* dcols, const int64_t* len_in, const float* relu_out, float* dX, int64_t B,
                      int64_t T1, int64_t F1, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dcols && dX, "null pointer");
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  const int64_t n = B * T1 * F1 * C;
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(col2im_kernel<false>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), dcols, len_in,
                     relu_out, dX, B, T1, F1, C, T2, F2);
  return check_launch("kdfm_col2im_3x3s2");
}

int kdfm_col2im_3x3s2_tapmajor(const float* dcols, const int64_t* len_in, const float* relu_out, float* dX, int64_t B,
                      int64_t T1, int64_t F1, int64_t C, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dcols && dX, "null pointer");
  const int64_t T2 = (T1 - 1) / 2 + 1, F2 = (F1 - 1) / 2 + 1;
  const int64_t n = B * T1 * F1 * C;
  if (n == 0) return KDFM_OK;
  hipLaunchKernelGGL(col2im_kernel<true>, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream), dcols, len_in,
                     relu_out, dX, B, T1, F1, C, T2, F2);
  return check_launch("kdfm_col2im_3x3s2_tapmajor");
}

}  // extern "C"
