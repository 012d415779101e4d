// Fused Conformer macaron FFN block (LayerNorm -> Linear(d,4d) -> SiLU -> dropout -> Linear(4d,d) ->
// dropout -> scaled residual), forward and data-gradient backward, one launch each (bf16 MFMA, f32
// state).
//
// Reference: ConformerLayer.forward, the two half-step feed-forward modules (SURVEY.md Appendix A.5,
// NeMo conformer_modules.py ConformerFeedForward; built conformer_encoder.py:450-472, called :685-692):
//   r_out = r_in + rscale * drop(W2 drop(silu(W1 LN(r_in) + b1)) + b2),   rscale = 0.5
// The unfused path ran LN, the up-projection (writing the 4d-wide pre-activation AND activation in
// f32) and the down-projection as three launches; here one wave keeps 32 rows of LN(r_in) as bf16
// MFMA operands in registers and streams the 4d hidden width through in 32-feature chunks, so the
// hidden activation never leaves the chip.  Training saves only the row statistics (mean, rstd); the
// backward recomputes the hidden chunk from LN(r_in) (same operands, same MFMA order: bit-identical
// to the forward's) and emits the bf16 weight-gradient operands ln, a, dl2, dh for kdfm_wgrad_bf16.
//
// Layout: every product is computed transposed, C^T (32 features x 32 rows) = W (32 x K) x X^T, with
// v_mfma_f32_32x32x16_bf16.  A operand: a fragment of a prepared weight image (kdfm_ffn_wprep:
// fragment-major, one 1 KB lane-contiguous block per (tile, k-step) -> conflict-free ds_read_b128),
// staged chunk by chunk through LDS and shared by the 4 waves of a workgroup.  B operand: the wave's
// rows, lane (r, h) holding 8 features k = 16 ks + 8 h .. +7 of row r.  The accumulator gives lane
// (r, h) the features 8 q + 4 h + 0..3 of row r; one v_permlane32_swap per packed bf16 dword turns a
// chunk's activation into the B operand of the next product (cdna_hip_programming.md T21).
//
// Work split: a workgroup owns 64 rows = 2 row tiles of 32.  Backward: NP = 2 waves per tile take the
// chunks c = NP it + par, their dLN partials added in a fixed order through LDS like the forward's.
// Forward (d <= 96): NP = 4 waves per tile take the chunks
// c = NP it + par, so 12,832 rows give 1,604 waves (the kernel is latency bound: a wave's serial
// chain of chunks sets the launch time and 201 workgroups fill at most 201 CUs); their partial
// down-projections are added in the fixed order ((p0 + p1) + p2) + p3 through LDS at the end, and
// registers are held to 256 per lane (launch bound 512) so the 8 waves run 2 per SIMD.  d = 176
// keeps NP = 2 (even / odd chunks, 256 threads).
#include "lnblock.h"
#include "wimg.h"

// timing probe points (tools/ffn_probe.hip defines FFN_PROBE; empty in the library)
#ifndef FFN_PROBE
#define FFN_PROBE(i)
#endif

namespace kdfm {
namespace {

using namespace lnb;

constexpr int FF_NT = 256;        // backward: 4 waves = 2 row tiles x 2 chunk parities
constexpr int FF_ROWS = 64;       // rows per workgroup
// forward: chunk parities per row tile (4 for d <= 96; d = 176 keeps 2: four 23 KB chunks per stage and
// its 96 accumulators do not fit the 256-register budget of 2 waves per SIMD)
template <int DT> constexpr int fwd_np() { return DT <= 3 ? 4 : 2; }
template <int DT> constexpr int fwd_nt() { return 2 * fwd_np<DT>() * 64; }
// backward: 2 chunk parities per row tile (4 waves).  Measured: 4 parities (8 waves, 144 KB of stages,
// the 256-register cap of 2 waves per SIMD) ran 67.6 us against 64.8 us per in-step launch
// (profiles/r03/r3f_kernel_summary.txt vs r3b): the shorter chain did not pay for the larger stages
template <int DT> constexpr int bwd_np() { return 2; }
template <int DT> constexpr int bwd_nt() { return 2 * bwd_np<DT>() * 64; }

// Chunk image (one 32-feature slice of the hidden width), fragment order:
//   W2c(mt, ks2) = 2 mt + ks2            A of the down-projection (d rows x 32 hidden)     [fwd]
//   W1c(ks)      = 2 DT + ks             A of the up-projection (32 hidden x d)            [fwd, bwd]
//   W2Tc(ks)     = 2 DT + KS1 + ks       A of dA^T = W2^T dl2^T (32 hidden x d)             [bwd]
//   W1Tc(mt,ks2) = 2 DT + 2 KS1 + 2 mt + ks2   A of dln^T = W1^T dh^T (d rows x 32 hidden)  [bwd]
// so the forward stages fragments [0, 2DT + KS1) and the backward [2DT, CS) of each chunk.
template <int KS1, int DT>
struct FfnGeo {
  static constexpr int FWD = 2 * DT + KS1;
  static constexpr int BWD = 2 * KS1 + 2 * DT;
  static constexpr int CS = 4 * DT + 2 * KS1;
};

// ---- weight images ------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ffn_wprep_kernel(const float* __restrict__ W1, const float* __restrict__ W2,
                                                        uint16_t* __restrict__ img, int d, int ff, int KS1, int DT,
                                                        int nfr, int64_t total) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  const int lane = (int)(g & 63);
  const int64_t rest = g >> 6;
  const int f = (int)(rest % nfr);
  const int64_t c = rest / nfr;
  float v[8];
  wimg::ffn_frag(W1, W2, d, ff, KS1, DT, c, f, lane, v);
  *reinterpret_cast<bf16x8*>(img + ((c * (4 * DT + 2 * KS1) + f) * 64 + lane) * 8) = pack_bf16x8<bf16x8>(v);
}

struct FfnFwd {
  const float* x; const float* g; const float* b; float eps;
  const uint16_t* img; const float* b1; const float* b2;
  float* out; float* mean; float* rstd;
  int64_t rows; int d, ff;
  float rscale, p_act, p_out;
  const uint64_t* seed; uint64_t st_act, st_out;
  // optional LayerNorm of the block output (the layer's norm_out after feed_forward2):
  // ln_out = LN(out) with (ln_g, ln_b, ln_eps); its row statistics to ln_mean / ln_rstd
  const float* ln_g; const float* ln_b; float ln_eps; float* ln_out; float* ln_mean; float* ln_rstd;
};

// bytes of the backward's weight-stage region (double-buffered NP-chunk stages, reused for the final
// reduction of the NP - 1 partials per tile); the per-feature vectors (biases) follow it in LDS: a global
// bias load inside the chunk loop would wait (in-order vmcnt) for the next stage's prefetch and expose
// its latency every iteration
template <int SF, int DT>
constexpr int ffn_stage_bytes() {
  constexpr int NP = bwd_np<DT>();
  return 2 * NP * SF * 1024 > 2 * (NP - 1) * DT * 16 * 64 * 4 ? 2 * NP * SF * 1024 : 2 * (NP - 1) * DT * 16 * 64 * 4;
}
// forward: two stages of NP chunks, or the NP - 1 partials per tile of the final reduction
template <int SF, int DT>
constexpr int ffn_fwd_stage_bytes() {
  constexpr int NP = fwd_np<DT>();
  return 2 * NP * SF * 1024 > 2 * (NP - 1) * DT * 16 * 64 * 4 ? 2 * NP * SF * 1024 : 2 * (NP - 1) * DT * 16 * 64 * 4;
}

template <int KS1, int DT>
__global__ __launch_bounds__(fwd_nt<DT>()) void ffn_fwd_kernel(FfnFwd a) {
  using G = FfnGeo<KS1, DT>;
  constexpr int FWD_NP = fwd_np<DT>(), FWD_NT = fwd_nt<DT>();
  extern __shared__ __attribute__((aligned(16))) uint4 ff_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, par = wave % FWD_NP, tile = wave / FWD_NP;
  const int64_t row = (int64_t)blockIdx.x * FF_ROWS + tile * 32 + (lane & 31);
  const bool ok = row < a.rows;
  const int d = a.d, ff = a.ff, FC = ff / 32;
  const uint64_t seed = (a.p_act > 0.f || a.p_out > 0.f) ? load_seed(a.seed) : 0ull;
  const uint64_t kact = rng_key(seed, a.st_act), kout = rng_key(seed, a.st_out);
  const float ks_act = 1.f / (1.f - a.p_act), ks_out = 1.f / (1.f - a.p_out);

  FFN_PROBE(0);
  using DS = DmaStager<G::FWD, 0, G::CS, FWD_NP, FWD_NT>;
  const uint4* img = reinterpret_cast<const uint4*>(a.img);
  DS::issue(img, 0, FC, ff_lds, 0);

  // prologue: the row loads, the bias / gamma / beta table fill and the stage-0 DMA are all in flight
  // together; one barrier; then the LayerNorm from registers and the LDS table
  float xv[KS1][8];
  ln_load<KS1>(a.x, row, ok, d, h, xv);
  float* bias_s = reinterpret_cast<float*>(reinterpret_cast<char*>(ff_lds) + ffn_fwd_stage_bytes<G::FWD, DT>());
  // [b1 | b2 | gamma | beta | (norm_out) gamma | beta]: ff = 4 d <= 4 * 32 DT
  const int nlo = a.ln_out ? d : 0;
  fill_vec6<9 * 32 * DT, FWD_NT>(bias_s, a.b1, ff, a.b2, d, a.g, d, a.b, d, a.ln_out ? a.ln_g : a.b, nlo,
                                 a.ln_out ? a.ln_b : a.b, nlo);
  f32x16 acc[DT];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;
  // the residual rows in the accumulator layout for the epilogue, fetched now so their latency hides
  // behind the chunk loop (narrow d only: 4 DT float4 registers)
  constexpr bool XPRE = DT <= 3 && FWD_NP == 2;
  float4 xres[DT][4];   // (wide d: loaded after the chunk loop, below)
  if constexpr (XPRE) {
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = mt * 32 + 8 * q + 4 * h;
        const bool in = par == 0 && ok && n0 < d;
        xres[mt][q] = *reinterpret_cast<const float4*>(a.x + (in ? row * d + n0 : 0));
      }
  }
  FFN_PROBE(1);
  __syncthreads();   // stage 0 landed, the tables written
  FFN_PROBE(2);
  float mean = 0.f, rstd = 0.f;
  bf16x8 bx[KS1];
  ln_finish<KS1>(xv, bias_s + ff + d, bias_s + ff + 2 * d, row, ok, d, h, a.eps, false, mean, rstd, bx, nullptr);
  // the row statistics as 2 buffer stores every lane issues (the lanes that own no statistic write past
  // the buffer, dropped)
  {
    const bool own = a.mean != nullptr && par == 0 && h == 0 && ok;
    const int nb = a.mean ? (int)(a.rows * 4) : 0;
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)a.mean, (short)0, nb, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)a.rstd, (short)0, nb, 0x00020000);
    const uint32_t off = own ? (uint32_t)(row * 4) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, mean), rm, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, rstd), rr, off, 0, 0);
  }
  const int nit = (FC + FWD_NP - 1) / FWD_NP;
  for (int it = 0; it < nit; ++it) {
    // no branch around the chunk (a conditional MFMA block makes the compiler carry acc through the
    // loop in VGPRs and copy it to and from AGPRs every iteration): a parity past the last chunk
    // computes on the clamped, loaded last block and adds an all-zero activation operand (+0 exactly)
    const int c = FWD_NP * it + par;
    const bool live = c < FC;
    // the chunk's biases are read from LDS BEFORE the next stage's DMA is issued: an LDS read while an
    // LDS-DMA is in flight makes the compiler drain it (vmcnt(0)) first
    float4 bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = *reinterpret_cast<const float4*>(bias_s + c * 32 + 8 * q + 4 * h);
    if (it + 1 < nit) DS::issue(img, it + 1, FC, ff_lds, (it + 1) & 1);
    {
      const uint4* W = DS::block(ff_lds, it & 1, par);
      f32x16 hacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) hacc[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks)
        hacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(W[(2 * DT + ks) * FRAG_U4 + lane]), bx[ks], hacc, 0, 0, 0);
      uint32_t pk[4][2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = c * 32 + 8 * q + 4 * h;
        const float bv[4] = {bq[q].x, bq[q].y, bq[q].z, bq[q].w};
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = siluf_(hacc[4 * q + i] + bv[i]);
        if (a.p_act > 0.f) {
          bool kp[4];
          dropout_keep2_k(kact, (uint64_t)row * ff + n0, a.p_act, kp[0], kp[1]);
          dropout_keep2_k(kact, (uint64_t)row * ff + n0 + 2, a.p_act, kp[2], kp[3]);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = kp[i] ? v[i] * ks_act : 0.f;
        }
        pk[q][0] = live ? pack_bf16x2(v[0], v[1]) : 0u;
        pk[q][1] = live ? pack_bf16x2(v[2], v[3]) : 0u;
      }
      bf16x8 ba[2];
      tile_operands(pk, ba);
#pragma unroll
      for (int mt = 0; mt < DT; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(W[(2 * mt + s) * FRAG_U4 + lane]), ba[s], acc[mt], 0, 0, 0);
    }
    FFN_PROBE(4 + 2 * it);
    __syncthreads();
    FFN_PROBE(5 + 2 * it);
  }
  // wide d (4 waves, 512 registers): the epilogue's residual rows, all issued before any of its stores
  // (one wait, not one per row piece behind the previous store) and before the partials' reduction so
  // their latency overlaps it
  if constexpr (!XPRE && DT > 3) {
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = mt * 32 + 8 * q + 4 * h;
        const bool in = par == 0 && ok && n0 < d;
        xres[mt][q] = *reinterpret_cast<const float4*>(a.x + (in ? row * d + n0 : 0));
      }
  }
  // partials of parities 1..NP-1 -> parity 0, added in the fixed order ((p0 + p1) + p2) + p3
  float* red = reinterpret_cast<float*>(ff_lds) + tile * ((FWD_NP - 1) * DT * 16 * 64);
  if (par != 0) {
    float* mine = red + (par - 1) * (DT * 16 * 64);
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mine[(mt * 16 + i) * 64 + lane] = acc[mt][i];
  }
  __syncthreads();
  FFN_PROBE(30);
  if (par != 0) return;   // (every lane of the parity-0 wave stays: the optional LN reduces across lanes)

#pragma unroll
  for (int q = 1; q < FWD_NP; ++q)
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][i] += red[((q - 1) * DT * 16 + mt * 16 + i) * 64 + lane];
  float o[DT][16];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = mt * 32 + 8 * q + 4 * h;
      const bool in = ok && n0 < d;
      const float4 bb = *reinterpret_cast<const float4*>(bias_s + ff + (n0 < d ? n0 : 0));
      // (narrow d: loaded here, one piece at a time -- batching them spills at 2 waves per SIMD)
      const float4 xr = (XPRE || DT > 3) ? xres[mt][q] : *reinterpret_cast<const float4*>(a.x + (in ? row * d + n0 : 0));
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w}, xv[4] = {xr.x, xr.y, xr.z, xr.w};
      bool kp[4] = {true, true, true, true};
      if (a.p_out > 0.f) {
        dropout_keep2_k(kout, (uint64_t)row * d + n0, a.p_out, kp[0], kp[1]);
        dropout_keep2_k(kout, (uint64_t)row * d + n0 + 2, a.p_out, kp[2], kp[3]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[mt][4 * q + i] + bv[i];
        if (a.p_out > 0.f) v = kp[i] ? v * ks_out : 0.f;
        o[mt][4 * q + i] = in ? xv[i] + a.rscale * v : 0.f;
      }
      if (in)
        *reinterpret_cast<float4*>(a.out + row * d + n0) =
            make_float4(o[mt][4 * q], o[mt][4 * q + 1], o[mt][4 * q + 2], o[mt][4 * q + 3]);
    }
  FFN_PROBE(31);
  if (!a.ln_out) return;
  asm volatile("" ::: "memory");   // keep the gamma / beta table reads below here (register pressure)
  // norm_out: two-pass row statistics (this lane's half of the row + its partner lane's)
  float s = 0.f;
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += o[mt][e];
  s += __shfl_xor(s, 32, 64);
  const float mu = s / d;
  float qv = 0.f;
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const bool in = mt * 32 + 8 * (e / 4) + 4 * h + (e % 4) < d;
      const float t = in ? o[mt][e] - mu : 0.f;
      qv += t * t;
    }
  qv += __shfl_xor(qv, 32, 64);
  const float rs = rsqrtf(qv / d + a.ln_eps);
  if (!ok) return;
  if (h == 0) {
    a.ln_mean[row] = mu;
    a.ln_rstd[row] = rs;
  }
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n0 = mt * 32 + 8 * q + 4 * h;
      if (n0 >= d) continue;
      const float4 gg = *reinterpret_cast<const float4*>(bias_s + ff + 3 * d + n0);   // LDS table
      const float4 bb = *reinterpret_cast<const float4*>(bias_s + ff + 4 * d + n0);
      const float gv[4] = {gg.x, gg.y, gg.z, gg.w}, bv[4] = {bb.x, bb.y, bb.z, bb.w};
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = (o[mt][4 * q + i] - mu) * rs * gv[i] + bv[i];
      *reinterpret_cast<float4*>(a.ln_out + row * d + n0) = make_float4(y[0], y[1], y[2], y[3]);
    }
}

struct FfnBwd {
  const float* dout; const float* x; const float* mean; const float* rstd; const float* g; const float* b;
  const uint16_t* img; const float* b1;
  float* dx; uint16_t* ln_h; uint16_t* a_h; uint16_t* dl2_h; uint16_t* dh_h; float* part;
  int64_t rows, nparts; int d, ff;
  float rscale, p_act, p_out;
  const uint64_t* seed; uint64_t st_act, st_out;
};

template <int KS1, int DT>
__global__ __launch_bounds__(bwd_nt<DT>()) void ffn_bwd_kernel(FfnBwd a) {
  using G = FfnGeo<KS1, DT>;
  constexpr int NP = bwd_np<DT>(), NT = bwd_nt<DT>();
  extern __shared__ __attribute__((aligned(16))) uint4 ff_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, par = wave % NP, tile = wave / NP;
  const int64_t row = (int64_t)blockIdx.x * FF_ROWS + tile * 32 + (lane & 31);
  const bool ok = row < a.rows;
  const int d = a.d, ff = a.ff, FC = ff / 32;
  const uint64_t seed = (a.p_act > 0.f || a.p_out > 0.f) ? load_seed(a.seed) : 0ull;
  const uint64_t kact = rng_key(seed, a.st_act), kout = rng_key(seed, a.st_out);
  const float ks_act = 1.f / (1.f - a.p_act), ks_out = 1.f / (1.f - a.p_out);

  using DS = DmaStager<G::BWD, 2 * DT, G::CS, NP, NT>;
  const uint4* img = reinterpret_cast<const uint4*>(a.img);
  DS::issue(img, 0, FC, ff_lds, 0);
  const int side_bytes = (int)(a.rows * ff * 2);
  const __amdgpu_buffer_rsrc_t r_a = __builtin_amdgcn_make_buffer_rsrc((void*)a.a_h, (short)0, side_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r_dh = __builtin_amdgcn_make_buffer_rsrc((void*)a.dh_h, (short)0, side_bytes, 0x00020000);

  // prologue loads first (row statistics, x rows, the bias / gamma / beta table, dout below): every load
  // is issued before the prologue's stores, so waiting for a load never waits for a store
  float mean = ok ? a.mean[row] : 0.f, rstd = ok ? a.rstd[row] : 0.f;
  float xv[KS1][8];
  ln_load<KS1>(a.x, row, ok, d, h, xv);
  float* bias_s = reinterpret_cast<float*>(reinterpret_cast<char*>(ff_lds) + ffn_stage_bytes<G::BWD, DT>());
  fill_vec5<6 * 32 * DT, NT>(bias_s, a.b1, ff, a.g, d, a.b, d, a.b, 0, a.b, 0);
  // dl2 = rscale * drop_out(dout): B operands of dA^T; the even wave writes the bf16 copy (dW2 operand)
  bf16x8 bd[KS1];
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const int k0 = ks * 16 + 8 * h;
    const bool in = ok && k0 < d;
    const float4* p = reinterpret_cast<const float4*>(a.dout + (in ? row * d + k0 : 0));
    const float4 u = p[0], w = p[1];
    float v[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
    bool kp[8] = {true, true, true, true, true, true, true, true};
    if (a.p_out > 0.f)
#pragma unroll
      for (int j = 0; j < 8; j += 2) dropout_keep2_k(kout, (uint64_t)row * d + k0 + j, a.p_out, kp[j], kp[j + 1]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = in ? v[j] * a.rscale : 0.f;
      if (a.p_out > 0.f) t = kp[j] ? t * ks_out : 0.f;
      v[j] = t;
    }
    bd[ks] = pack_bf16x8<bf16x8>(v);
  }
  __syncthreads();   // stage 0 landed, the tables written
  bf16x8 bx[KS1];
  ln_finish<KS1>(xv, bias_s + ff, bias_s + ff + d, row, ok, d, h, 0.f, true, mean, rstd, bx, nullptr);
  // the bf16 copies of dl2 and LN(x) (weight-gradient operands): 2 KS1 buffer stores every lane issues
  // (other parities / rows past the end / features past d write past the buffer, dropped) -- a fixed
  // count for the counted barrier
  {
    const int rb = (int)(a.rows * d * 2);
    const __amdgpu_buffer_rsrc_t r_l2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.dl2_h, (short)0, rb, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_ln = __builtin_amdgcn_make_buffer_rsrc((void*)a.ln_h, (short)0, rb, 0x00020000);
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const int k0 = ks * 16 + 8 * h;
      const uint32_t off = (par == 0 && ok && k0 < d) ? (uint32_t)((row * d + k0) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, bd[ks]), r_l2, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, bx[ks]), r_ln, off, 0, 0);
    }
  }

  f32x16 acc[DT];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mt][i] = 0.f;


  const int nit = (FC + NP - 1) / NP;
  for (int it = 0; it < nit; ++it) {
    // branch-free chunk (as the forward): a parity past the last chunk adds an all-zero dh operand
    // and stores nothing; its biases are read before the next stage's DMA is issued
    const int c = NP * it + par;
    const bool live = c < FC;
    float4 bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = *reinterpret_cast<const float4*>(bias_s + (live ? c * 32 : 0) + 8 * q + 4 * h);
    if (it + 1 < nit) DS::issue(img, it + 1, FC, ff_lds, (it + 1) & 1);
    {
      const uint4* W = DS::block(ff_lds, it & 1, par);   // W1c | W2Tc | W1Tc
      f32x16 hacc, gacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) hacc[i] = gacc[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        hacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(W[ks * FRAG_U4 + lane]), bx[ks], hacc, 0, 0, 0);
        gacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(W[(KS1 + ks) * FRAG_U4 + lane]), bd[ks], gacc, 0, 0, 0);
      }
      uint32_t pa[4][2], pd[4][2];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n0 = c * 32 + 8 * q + 4 * h;
        const float bv[4] = {bq[q].x, bq[q].y, bq[q].z, bq[q].w};
        float av[4], dv[4];
        bool kq[4] = {true, true, true, true};
        if (a.p_act > 0.f) {
          dropout_keep2_k(kact, (uint64_t)row * ff + n0, a.p_act, kq[0], kq[1]);
          dropout_keep2_k(kact, (uint64_t)row * ff + n0 + 2, a.p_act, kq[2], kq[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float hv = hacc[4 * q + i] + bv[i];
          const float sg = sigmoidf_(hv);
          float s = hv * sg, gv = gacc[4 * q + i];
          if (a.p_act > 0.f) {
            s = kq[i] ? s * ks_act : 0.f;
            gv = kq[i] ? gv * ks_act : 0.f;
          }
          av[i] = s;
          dv[i] = gv * (sg * (1.f + hv * (1.f - sg)));
        }
        pa[q][0] = pack_bf16x2(av[0], av[1]);
        pa[q][1] = pack_bf16x2(av[2], av[3]);
        pd[q][0] = live ? pack_bf16x2(dv[0], dv[1]) : 0u;
        pd[q][1] = live ? pack_bf16x2(dv[2], dv[3]) : 0u;
      }
      bf16x8 ba[2], bdh[2];
      tile_operands(pa, ba);
      tile_operands(pd, bdh);
      // the four bf16 side-output stores are issued by every lane (rows past the end / a parity past the
      // last chunk carry an out-of-range offset the buffer range check drops): a fixed count behind the
      // stage's DMA for the counted barrier below
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t off = (ok && live) ? (uint32_t)((row * ff + c * 32 + s * 16 + 8 * h) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, ba[s]), r_a, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, bdh[s]), r_dh, off, 0, 0);
      }
#pragma unroll
      for (int mt = 0; mt < DT; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(W[(2 * KS1 + 2 * mt + s) * FRAG_U4 + lane]), bdh[s],
                                                            acc[mt], 0, 0, 0);
    }
    dma_barrier<4>();   // stage it + 1 landed; this iteration's 4 side-output stores stay in flight
  }
  // partials of parities 1..NP-1 -> parity 0, added in the fixed order ((p0 + p1) + p2) + p3
  float* red = reinterpret_cast<float*>(ff_lds) + tile * ((NP - 1) * DT * 16 * 64);
  if (par != 0) {
    float* mine = red + (par - 1) * (DT * 16 * 64);
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mine[(mt * 16 + i) * 64 + lane] = acc[mt][i];
  }
  __syncthreads();
  if (par != 0) return;
  float dl[DT * 16];
#pragma unroll
  for (int mt = 0; mt < DT; ++mt)
#pragma unroll
    for (int e = 0; e < 16; ++e) dl[mt * 16 + e] = acc[mt][e];
#pragma unroll
  for (int q = 1; q < NP; ++q)
#pragma unroll
    for (int mt = 0; mt < DT; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) dl[mt * 16 + e] += red[((q - 1) * DT * 16 + mt * 16 + e) * 64 + lane];
  ln_backward_rows<DT>(dl, a.x, bias_s + ff, a.dout, a.dx, a.part, a.nparts, (int64_t)blockIdx.x * FF_ROWS + tile * 32, row, ok,
                       d, mean, rstd, lane);
}

int ffn_dims(int64_t d, int& KS1, int& DT) { return ln_dims(d, KS1, DT); }

template <typename K>
void ffn_allow_lds(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int KS1, int DT>
int launch_fwd(const FfnFwd& a, hipStream_t st) {
  using G = FfnGeo<KS1, DT>;
  static bool once = (ffn_allow_lds(ffn_fwd_kernel<KS1, DT>), true);
  (void)once;
  const size_t lds = (size_t)ffn_fwd_stage_bytes<G::FWD, DT>() + (size_t)(a.ff + 5 * a.d) * 4;
  if (lds > 160 * 1024) { set_error("kdfm_ffn_fwd: hidden width too large for the LDS bias table"); return KDFM_EINVAL; }
  hipLaunchKernelGGL((ffn_fwd_kernel<KS1, DT>), dim3((unsigned)ceil_div(a.rows, FF_ROWS)), dim3(fwd_nt<DT>()), lds, st, a);
  return check_launch("kdfm_ffn_fwd");
}

template <int KS1, int DT>
int launch_bwd(const FfnBwd& a, hipStream_t st) {
  using G = FfnGeo<KS1, DT>;
  static bool once = (ffn_allow_lds(ffn_bwd_kernel<KS1, DT>), true);
  (void)once;
  const size_t lds = (size_t)ffn_stage_bytes<G::BWD, DT>() + (size_t)(a.ff + 2 * a.d) * 4;
  hipLaunchKernelGGL((ffn_bwd_kernel<KS1, DT>), dim3((unsigned)ceil_div(a.rows, FF_ROWS)), dim3(bwd_nt<DT>()), lds, st,
                     a);
  return check_launch("kdfm_ffn_bwd");
}

}  // namespace
}  // namespace kdfm

extern "C" {

int32_t kdfm_ffn_supported(int64_t d, int64_t ff) {
  int KS1, DT;
  return kdfm::ffn_dims(d, KS1, DT) == 0 && ff > 0 && ff % 32 == 0 && ff <= 128 * DT ? 1 : 0;
}

int64_t kdfm_ffn_img_elems(int64_t d, int64_t ff) {
  int KS1, DT;
  if (kdfm::ffn_dims(d, KS1, DT) != 0 || ff <= 0 || ff % 32 != 0) return 0;
  return (ff / 32) * (int64_t)(4 * DT + 2 * KS1) * 512;
}

int kdfm_ffn_wprep(const float* W1, const float* W2, uint16_t* img, int64_t d, int64_t ff, int32_t fwd_only,
                   void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(W1 && W2 && img, "null pointer");
  int KS1, DT;
  KDFM_REQUIRE(ffn_dims(d, KS1, DT) == 0 && ff > 0 && ff % 32 == 0 && ff <= 128 * DT, "unsupported FFN shape (d, ff)");
  KDFM_REQUIRE(al16(img), "img must be 16-byte aligned");
  const int CS = 4 * DT + 2 * KS1;
  const int nfr = fwd_only ? 2 * DT + KS1 : CS;
  const int64_t total = (ff / 32) * (int64_t)nfr * 64;
  hipLaunchKernelGGL(ffn_wprep_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, as_stream(stream), W1, W2,
                     img, (int)d, (int)ff, KS1, DT, nfr, total);
  return check_launch("kdfm_ffn_wprep");
}

int kdfm_ffn_fwd(const float* x, const float* ln_g, const float* ln_b, float ln_eps, const uint16_t* img,
                 const float* b1, const float* b2, float* out, float* mean, float* rstd, int64_t rows, int64_t d,
                 int64_t ff, float rscale, float p_act, float p_out, const uint64_t* seed, uint64_t stream_act,
                 uint64_t stream_out, const float* out_ln_g, const float* out_ln_b, float out_ln_eps, float* out_ln,
                 float* out_ln_mean, float* out_ln_rstd, void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(x && ln_g && ln_b && img && b1 && b2 && out, "null pointer");
  KDFM_REQUIRE((mean == nullptr) == (rstd == nullptr), "mean and rstd go together");
  int KS1, DT;
  KDFM_REQUIRE(ffn_dims(d, KS1, DT) == 0 && ff > 0 && ff % 32 == 0 && ff <= 128 * DT, "unsupported FFN shape (d, ff)");
  KDFM_REQUIRE(al16(x) && al16(out) && al16(ln_g) && al16(ln_b) && al16(b1) && al16(b2) && al16(img),
               "operands must be 16-byte aligned");
  KDFM_REQUIRE(p_act >= 0.f && p_act < 1.f && p_out >= 0.f && p_out < 1.f, "dropout p");
  KDFM_REQUIRE((p_act == 0.f && p_out == 0.f) || seed, "dropout needs a seed");
  if (rows <= 0) return KDFM_OK;
  KDFM_REQUIRE(!out_ln || (out_ln_g && out_ln_b && out_ln_mean && out_ln_rstd && al16(out_ln) && al16(out_ln_g) &&
                             al16(out_ln_b)),
               "output LayerNorm needs gamma / beta / mean / rstd (16-byte aligned)");
  FfnFwd a{x, ln_g, ln_b, ln_eps, img, b1, b2, out, mean, rstd, rows, (int)d, (int)ff, rscale, p_act, p_out,
           seed, stream_act, stream_out, out_ln_g, out_ln_b, out_ln_eps, out_ln, out_ln_mean, out_ln_rstd};
  hipStream_t st = as_stream(stream);
  if (KS1 == 6) return launch_fwd<6, 3>(a, st);
  if (KS1 == 11) return launch_fwd<11, 6>(a, st);
  return launch_fwd<12, 6>(a, st);
}

int kdfm_ffn_bwd(const float* dout, const float* x, const float* mean, const float* rstd, const float* ln_g,
                 const float* ln_b, const uint16_t* img, const float* b1, float* dx, uint16_t* ln_h, uint16_t* a_h,
                 uint16_t* dl2_h, uint16_t* dh_h, float* part, int64_t rows, int64_t d, int64_t ff, float rscale,
                 float p_act, float p_out, const uint64_t* seed, uint64_t stream_act, uint64_t stream_out,
                 void* stream) {
  using namespace kdfm;
  KDFM_REQUIRE(dout && x && mean && rstd && ln_g && ln_b && img && b1 && dx && ln_h && a_h && dl2_h && dh_h && part,
               "null pointer");
  int KS1, DT;
  KDFM_REQUIRE(ffn_dims(d, KS1, DT) == 0 && ff > 0 && ff % 32 == 0 && ff <= 128 * DT, "unsupported FFN shape (d, ff)");
  KDFM_REQUIRE(al16(dout) && al16(x) && al16(dx) && al16(ln_g) && al16(ln_b) && al16(b1) && al16(img) &&
                   al16(ln_h) && al16(a_h) && al16(dl2_h) && al16(dh_h),
               "operands must be 16-byte aligned");
  KDFM_REQUIRE(p_act >= 0.f && p_act < 1.f && p_out >= 0.f && p_out < 1.f, "dropout p");
  KDFM_REQUIRE((p_act == 0.f && p_out == 0.f) || seed, "dropout needs a seed");
  KDFM_REQUIRE(rows * ff * 2 <= (int64_t)INT32_MAX - 64, "rows x ff exceeds the 2 GB side-output buffer range");
  if (rows <= 0) return KDFM_OK;
  FfnBwd a{dout, x, mean, rstd, ln_g, ln_b, img, b1, dx, ln_h, a_h, dl2_h, dh_h, part, rows, ceil_div(rows, 16),
           (int)d, (int)ff, rscale, p_act, p_out, seed, stream_act, stream_out};
  hipStream_t st = as_stream(stream);
  if (KS1 == 6) return launch_bwd<6, 3>(a, st);
  if (KS1 == 11) return launch_bwd<11, 6>(a, st);
  return launch_bwd<12, 6>(a, st);
}

}  // extern "C"
