/*
 * kdfm.h — C-ABI of libkdfm.so, the MI355X (gfx950) kernels of the ver5 flow-matching
 * distillation training step of qwer55252/KD-via-FM-in-ASR (asr_train_diffm.py).
 *
 * The reference has no native boundary on this path: every op is a torch/ATen call made from
 * NeMo modules.  This header is the boundary the build introduces beneath the
 * NeMo-signature Python modules in kd-via-fm-in-asr_amd/kdfm/.  Each entry point names, in its
 * comment, the reference call site whose arithmetic it replaces.
 *
 * Conventions (all entry points):
 *   - plain device pointers, int64 sizes/strides in ELEMENTS, caller's hipStream_t as void*;
 *   - the caller allocates every output and workspace; the library never allocates or frees;
 *   - calls are stream-ordered, never synchronise the host, and are safe to capture in a graph;
 *   - return 0 (KDFM_OK) or a kdfm_status; kdfm_last_error() gives a thread-local message;
 *   - tensors are fp32 unless stated; `mode` selects the MFMA arithmetic (see kdfm_math).
 */
#ifndef KDFM_H_
#define KDFM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum kdfm_status {
  KDFM_OK = 0,
  KDFM_EINVAL = 1,   /* bad shape / stride / pointer */
  KDFM_ELAUNCH = 2,  /* hipLaunch / hipGetLastError failure */
  KDFM_EUNSUPPORTED = 3
} kdfm_status;

typedef enum kdfm_math {
  KDFM_MATH_F32 = 0,  /* exact f32 MFMA (v_mfma_f32_16x16x4_f32): parity mode            */
  KDFM_MATH_BF16 = 1  /* bf16 operands, f32 accumulate (v_mfma_f32_16x16x32_bf16)       */
} kdfm_math;

/* library identity */
const char* kdfm_version(void);
const char* kdfm_last_error(void);
int kdfm_device_arch(char* buf, int64_t len); /* writes the gcnArchName of the current device */
/* Deterministic-reduction mode ("a deterministic reduction flag is used for parity
 * runs").  When on, every reduction that feeds an activation or a gradient runs in a fixed order:
 * GEMM split-K and batch-axis reductions become ordered launches, per-block partial folds
 * (column sums, BatchNorm statistics and their backward, NoiseAdapter gate gradients) run in one
 * workgroup per output group, wide-tile weight-gradient partials fold in slab order — so two runs
 * on the same inputs give bitwise-identical activations and gradients.  Scalar loss accumulators
 * (MSE / KL sums) keep float atomics and may differ in the last bits.  Process-global; read on the
 * host when a launch is configured (set it before capturing a graph).  Default off. */
void kdfm_set_deterministic(int32_t on);
int32_t kdfm_get_deterministic(void);

/* Tracing (the reference's Lightning profiler / NVTX ranges): a ROCTx range on the
 * calling host thread, seen by `rocprofv3 --marker-trace` next to the kernels it enqueued.
 * push returns the 0-based nesting level of the range it opened; pop returns the level of the range
 * it closed (negative if none was open). */
int32_t kdfm_range_push(const char* name);
int32_t kdfm_range_pop(void);

/* Step-plan replay primitives (kdfm/plan.py records one training step's launches and re-issues them
 * without the Python wrappers): hipEventRecord(event, stream), hipStreamWaitEvent(stream, event, 0)
 * and hipMemsetAsync on the caller's handles; they exist so a replay uses the same HIP runtime as the
 * kernels.  `event` is a hipEvent_t, `stream` a hipStream_t, both owned by the caller. */
int kdfm_event_record(void* event, void* stream);
int kdfm_stream_wait_event(void* stream, void* event);
/* Cross-stream link events: *event = a hipEvent_t created with hipEventDisableTiming | flags (flags: the HIP
 * release-scope flags, e.g. hipEventReleaseToDevice 0x40000000 or hipEventDisableSystemFence 0x20000000 -- a
 * link between two streams of one device needs no system-scope fence); destroy with kdfm_event_destroy. */
int kdfm_event_create(void** event, uint32_t flags);
int kdfm_event_destroy(void* event);
/* A HIP stream restricted to n_cus CUs spread uniformly over the device (hipExtStreamCreateWithCUMask);
 * *out receives the hipStream_t (the caller destroys it with hipStreamDestroy). */
int kdfm_stream_create_cu_mask(int32_t n_cus, void** out);
int kdfm_memset_async(void* ptr, int32_t value, int64_t bytes, void* stream);

/* --------------------------------------------------------------------------------------------
 * Generic batched GEMM with fused epilogue:
 *   C[b](m,n) = epi( alpha * sum_k A[b](m,k) * B[b](k,n) )
 * Replaces every nn.Linear / 1x1 Conv1d / Conv1d(k=3) / matmul on the path:
 *   Conformer FFN + attention projections (NeMo asr/parts ConformerLayer, called from
 *   conformer_encoder.py:685-692), ConvASRDecoder (conv_asr.py:445-468), KD heads
 *   (asr_train_diffm.py:400-460, 1295-1338), the STFT-as-DFT and mel matmul of the frontend
 *   (audio_preprocessing.py:299-300) and all of their backward products.
 * Element addressing: A(m,k) = A + b1*bA1 + b2*bA2 + m*sAm + k*sAk (likewise B, C, R, aux, Cpre).
 * conv3 modes: amode/bmode = KDFM_LD_CONV computes a 1-D convolution along the frame axis:
 *   A(m,k) with k = tap*conv_c + c reads row (m + tap - conv_pad) of a [rows][conv_c] matrix,
 *   zero outside the utterance (rows grouped in runs of conv_t frames). bmode CONV: same with
 *   the row index being k and the column n = tap*conv_c + c.
 * ------------------------------------------------------------------------------------------ */
typedef enum kdfm_ld {
  KDFM_LD_KC = 0,  /* operand contiguous along k (A row-major / B as W[n][k])  */
  KDFM_LD_XC = 1,  /* operand contiguous along m (A) or n (B)                  */
  KDFM_LD_CONV = 2 /* k = tap*conv_c + c, shifted-row gather (see above)        */
} kdfm_ld;

enum {
  KDFM_EPI_BIAS = 1 << 0,      /* += bias[n]                                            */
  KDFM_EPI_STORE_PRE = 1 << 1, /* Cpre = value after bias (pre-activation)              */
  KDFM_EPI_RELU = 1 << 2,      /* act = relu                                            */
  KDFM_EPI_SILU = 1 << 3,      /* act = silu                                            */
  KDFM_EPI_DROPOUT = 1 << 4,   /* inverted dropout, mask = rng(seed, stream, idx)       */
  KDFM_EPI_DRELU = 1 << 5,     /* *= relu'(aux)                                         */
  KDFM_EPI_DSILU = 1 << 6,     /* *= silu'(aux)                                         */
  KDFM_EPI_RESID = 1 << 7,     /* value = R + rscale*value   (R laid out like C)        */
  KDFM_EPI_BETA = 1 << 8,      /* value += beta*C_old                                   */
  KDFM_EPI_ATOMIC = 1 << 9,    /* atomicAdd into C (split-K reductions; no other epi)   */
  KDFM_EPI_ROWMASK = 1 << 10,  /* value = 0 on padded frames (see mask_len below)       */
  KDFM_EPI_MSE = 1 << 11       /* diff = value - R; C = rscale*diff; *loss_acc += loss_scale*diff^2 */
};

typedef struct kdfm_gemm_desc {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  const float* R;
  const float* aux;
  float* Cpre;
  int64_t M, N, K;
  int64_t sAm, sAk, sBk, sBn, sCm, sCn;
  int64_t batch1, batch2;
  int64_t bA1, bA2, bB1, bB2, bC1, bC2;
  float alpha, beta, rscale, dropout_p;
  const uint64_t* seed; /* device pointer, read at run time (graph-replay safe) */
  uint64_t rng_stream;
  int32_t amode, bmode, epi, math;
  int32_t splitk;
  int32_t conv_taps, conv_pad;
  int64_t conv_c, conv_t;
  /* EPI_ROWMASK: row m is frame t = (m / mask_div) % mask_T of utterance u = m / (mask_div*mask_T);
   * the value is zeroed when t >= mask_len[u] (NeMo pad_mask semantics). */
  const int64_t* mask_len;
  int64_t mask_T, mask_div;
  /* EPI_MSE accumulator (device scalar) */
  float* loss_acc;
  float loss_scale;
  /* implicit ones column (bias gradients fused into weight-gradient GEMMs): when ones_col >= 0,
   * B(k, ones_col) = 1 for every k (B memory holds only ones_col columns) and output column
   * ones_col is atomically added into ones_out[m] instead of C.  Requires EPI_ATOMIC. */
  float* ones_out;
  int64_t ones_col;
  /* optional device workspace (f32 elements): lets bf16 weight-gradient GEMMs (amode XC, EPI_ATOMIC,
   * K >> M*N) run as one wide-tile pass per row chunk with deterministic partial folding instead
   * of split-K atomics.  NULL / too small -> generic path.  kdfm_gemm_ws() gives the size used. */
  float* ws;
  int64_t ws_len;
  /* optional bf16 twin of the B operand (bf16 math only): B(k, n) ~= Bh[n*sBh + k], one row per
   * output column, contiguous along k — a weight's [out][in] layout for forward products or its
   * transpose for data gradients (kdfm_cast_bf16 / kdfm_cast_bf16_t build them once per step).
   * When set, skinny products stream B fragments straight from it instead of staging f32 weights
   * through LDS in every workgroup.  NULL: not used. */
  const uint16_t* Bh;
  int64_t sBh;
} kdfm_gemm_desc;

int kdfm_gemm(const kdfm_gemm_desc* d, void* stream);

/* Large-tile bf16 GEMM (csrc/biggemm.hip) for the wide layer products (d_model >= 512: the Conformer-large /
 * FastConformer(-XL) Linear layers, conformer_encoder.py:450-472 built at fast-conformer_ctc_bpe.yaml:29 widths),
 * replacing kdfm_gemm's generic 64x64 route for them.  bf16 operands in HBM, f32 accumulation:
 *   C[m][n] = epi(alpha * sum_k A(m, k) B(k, n)),  M x N x K from the descriptor,
 *   layout KDFM_BIG_NT: A(m, k) = A[m * lda + k], B(k, n) = B[n * ldb + k]   (forward: x W^T)
 *          KDFM_BIG_NN: A(m, k) = A[m * lda + k], B(k, n) = B[k * ldb + n]   (data gradient: dY W)
 *          KDFM_BIG_TN: A(m, k) = A[k * lda + m], B(k, n) = B[k * ldb + n]   (weight gradient: dY^T X)
 * The descriptor supplies C / strides and the epilogue (every kdfm_gemm flag except MSE, and at most one side
 * operand); C16 != NULL writes bf16 C16[m * sCm + n * sCn] instead of C.  epi == KDFM_EPI_ATOMIC means
 * ACCUMULATE: C += alpha * result, and ones_out[m] += alpha * sum_k A(m, k) when ones_out is set (the bias
 * gradient) -- one writer per element, fixed summation order (deterministic, unlike kdfm_gemm's split-K).
 * A, B 16-byte aligned, lda / ldb multiples of 8; kdfm_gemm_big_supported(M, N, K, layout) says whether the
 * shape is taken (M, N, K >= 64; k-contiguous operands: K % 8 == 0, the tail k-step zeroes the chunks past K;
 * k-major operands: their row length % 8 == 0). */
#define KDFM_BIG_NT 0
#define KDFM_BIG_NN 1
#define KDFM_BIG_TN 2
int kdfm_gemm_big_supported(int64_t M, int64_t N, int64_t K, int layout);
/* Workspace floats (descriptor ws / ws_len) the TN layout uses to split its reduction when the output tiles alone
 * cannot fill the chip (raw per-split partials folded in split order: still deterministic); 0 = no split.  Without
 * a large enough ws the product runs unsplit. */
int64_t kdfm_gemm_big_ws(int64_t M, int64_t N, int64_t K, int layout);
int kdfm_gemm_big(const kdfm_gemm_desc* d, const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int layout,
                  uint16_t* C16, void* stream);
/* fp8 e4m3 (OCP) products for FastConformer-XL at fp8 (BASELINE.json configs[4]: "fp8 MFMA attention/FFN"), MX
 * block scaling: every 32 consecutive elements along the contraction share one e8m0 scale byte (2^(byte - 127)).
 * kdfm_fp8_quant_mx: quantise a rows x cols f32 (src_bf16 = 0) or bf16 (1) matrix with row stride ld; the blocks run
 * along cols (transpose = 0: dst[r * ldd + c]) or along rows with the output transposed (transpose = 1: dst[c * ldd +
 * r], the data gradient's W^T); block exponent e = ceil(log2(amax / 448)), q = e4m3(x 2^-e) (no saturation), scale
 * byte e + 127, stored stage-major: scales[((k / 128) * R + row) * 4 + (k / 32) % 4] for output row `row` of R and
 * contraction index k.  The contraction length % 128 == 0.
 * kdfm_gemm_big_fp8: the KDFM_BIG_NT product (A(m, k) = A[m * lda + k], B(k, n) = B[n * ldb + k], byte strides) of
 * MX-quantised operands on the block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate; the
 * scales are applied by the MFMA) with the descriptor's epilogue; K % 128 == 0, M and N multiples of 4.  The
 * forward x W^T and the data gradient dY (W^T)^T (B = W quantised transposed) take it; weight gradients stay bf16. */
int kdfm_fp8_quant_mx(const void* src, int src_bf16, int64_t rows, int64_t cols, int64_t ld, uint8_t* dst, int64_t ldd,
                      uint8_t* scales, int transpose, void* stream);
int kdfm_gemm_big_fp8(const kdfm_gemm_desc* d, const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb,
                      const uint8_t* sa, const uint8_t* sb, uint16_t* C16, void* stream);
/* dst[r * ldd + c] = bf16(src[r * lds + c]) for a rows x cols f32 matrix (cols, lds, ldd multiples of 4). */
int kdfm_cast_bf16_2d(const float* src, int64_t lds, uint16_t* dst, int64_t ldd, int64_t rows, int64_t cols,
                      void* stream);

/* Row-parallel weight gradient with bf16 operands (the fused KD-head chains' saved operands):
 *   dW[m][n] += alpha * sum_r dY[r][m] * X[r][n]  (dW row stride ldc),  db[m] += alpha * sum_r dY[r][m]
 * dY (rows, M), X (rows, N) bf16 row-major, M % 4 == N % 4 == 0, 16-byte aligned; db may be NULL.
 * Per-workgroup partials in ws (kdfm_wgrad_bf16_ws floats, -1: shape unsupported) folded in a
 * fixed order (deterministic). */
int64_t kdfm_wgrad_bf16_ws(int64_t rows, int64_t M, int64_t N, int32_t bias);
int kdfm_wgrad_bf16(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                    int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len, void* stream);
/* Two weight gradients of the SAME shape in one launch (paired): dW (+)= alpha dY^T X and dW2 (+)= alpha
 * dY2^T X2 (+ db / db2 column sums, both or neither), one grid of 2x the single launch's workgroups and one
 * fold launch -- each product bitwise equal to its own kdfm_wgrad_bf16.  Used for the Conformer layer's
 * same-shape products (feed_forward1/2 linear1 and linear2, linear_out with pointwise_conv2): half the
 * launches on the weight-gradient stream.  ws >= 2 * kdfm_wgrad_bf16_ws(rows, M, N, bias) floats. */
int kdfm_wgrad_bf16_pair(const uint16_t* dY, const uint16_t* X, float* dW, float* db, const uint16_t* dY2,
                         const uint16_t* X2, float* dW2, float* db2, int64_t ldc, int64_t rows, int64_t M, int64_t N,
                         float alpha, float* ws, int64_t ws_len, void* stream);
/* The same over nseg = rows / seg_rows stacked segments (seg_rows % 32 == 0, nseg <= 16) with one bias
 * gradient per segment: db[j][m] += alpha * sum_{r in segment j} dY[r][m] (db is (nseg, M), required),
 * dW summed over all rows -- the FM chain's first-layer weight over its S steps in one launch
 * (asr_train_diffm.py:1368-1427: W1 is shared by the steps, the time-conditioned bias is per step). */
/* The same with the row count decided on the device: rows_dev[0] (<= rows, the capacity the launch and
 * the workspace are planned for, kdfm_wgrad_bf16_ws(rows, ...)) rows take part; read at run time, so a
 * producer kernel earlier on the stream may set it (kdfm_encfm_strategy's compact step saves). */
int kdfm_wgrad_bf16_dev(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                        const int64_t* rows_dev, int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len,
                        void* stream);
int64_t kdfm_wgrad_bf16_seg_ws(int64_t rows, int64_t M, int64_t N, int64_t seg_rows);
int kdfm_wgrad_bf16_seg(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t seg_rows,
                        int64_t rows, int64_t M, int64_t N, float alpha, float* ws, int64_t ws_len, void* stream);
/* The same for a Conv1d(C -> M, taps, padding pad) over utterances of T frames (rows % T == 0):
 *   dW[m][tap*C + c] += alpha * sum_r dY[r][m] * X[r + tap - pad][c]   (0 outside the utterance)
 * in the GEMM weight layout of kdfm_convw_prep (re-laid out by kdfm_convw_grad); the weight gradient
 * of SimpleDenoiser's convs (asr_train_diffm.py:449-453) over the fused chain's stacked saves. */
int64_t kdfm_wgrad_bf16_conv_ws(int64_t rows, int64_t M, int64_t C, int32_t taps, int32_t pad, int64_t T, int32_t bias);
int kdfm_wgrad_bf16_conv(const uint16_t* dY, const uint16_t* X, float* dW, int64_t ldc, float* db, int64_t rows,
                         int64_t M, int64_t C, int32_t taps, int32_t pad, int64_t T, float alpha, float* ws,
                         int64_t ws_len, void* stream);
/* The striding subsampling's second conv (Conv2d(C, C, 3, stride 2, padding 1), conformer_encoder.py:381-390,
 * subsampling.py ConvSubsampling) weight gradient straight from its bf16 input, no column matrix:
 *   dW[m][tap*C + c] += alpha * sum_{b,t2,f2} dY[(b,t2,f2)][m] * X[b][2 t2 - 1 + tap / 3][2 f2 - 1 + tap % 3][c]
 *   db[m] += alpha * sum dY[.][m]
 * X (B, T1, F1, C) bf16 channels-last, zero outside it and (len_in != NULL) at frames >= len_in[b];
 * dY (B*T2*F2, C) bf16, T2 = (T1-1)/2+1, F2 = (F1-1)/2+1; dW (C, 9C) tap-major (kdfm_convw_grad re-lays it
 * out).  The same sums, split plan and fold order as kdfm_wgrad_bf16 over kdfm_im2col_3x3s2_tm_from_bf16's
 * columns (bitwise equal), without the column matrix's 9/4 x |X| write and read.  C % 8 == 0, F1 >= 7;
 * ldx: X's row stride in elements (a multiple of 8, >= C; kdfm_subsample_fused's padded y1 rows);
 * ws: kdfm_wgrad_bf16_s2conv_ws floats (deferred folds apply). */
int64_t kdfm_wgrad_bf16_s2conv_ws(int64_t B, int64_t T1, int64_t F1, int64_t C);
int kdfm_wgrad_bf16_s2conv(const uint16_t* dY, const uint16_t* X, int64_t ldx, const int64_t* len_in, float* dW,
                           float* db, int64_t B, int64_t T1, int64_t F1, int64_t C, float alpha, float* ws,
                           int64_t ws_len, void* stream);
/* Deferred folds of the row-parallel weight gradients (kdfm_wgrad_bf16 / _pair / _seg / _conv / _dev), per
 * stream: after kdfm_wgrad_set_fold_arena(stream, arena, len) the products issued on `stream` write their
 * per-split partials into `arena` (len floats, caller-owned, 16-byte aligned; ws is then unused) and queue
 * their ordered fold instead of launching it; kdfm_wgrad_fold_flush(stream) folds every queued product in one
 * launch (up to 24 per launch), each exactly as its own fold would (bitwise equal gradients), and frees the
 * arena for the stream's next products (stream order).  dW / db are final only after the flush.  A product
 * whose partials do not fit the arena's remaining space folds at once as usual; queued products adding into
 * overlapping gradient memory fold in queue order (separate launches).  arena = NULL ends deferral
 * (the queue must be empty).  kdfm_wgrad_fold_pending: queued folds of the stream.  kdfm_wgrad_fold_stats:
 * out3 = [queued folds, products that did not fit the arena and folded at once since it was set, the largest
 * arena in floats the queue between two flushes would have needed] (host state, no device sync).
 * kdfm_wgrad_fold_discard_all: error recovery -- drop every stream's queued folds (their gradients are then
 * incomplete) and unset every arena; returns the number of jobs dropped. */
int kdfm_wgrad_set_fold_arena(void* stream, float* arena, int64_t len);
int kdfm_wgrad_fold_flush(void* stream);
int64_t kdfm_wgrad_fold_pending(void* stream);
int kdfm_wgrad_fold_stats(void* stream, int64_t* out3);
int kdfm_wgrad_fold_discard_all(void);

/* Fused FlowMatchingModule chain (asr_train_diffm.py:1368-1427, rectified, meta_encoder 'mlp',
 * shape_transform 'linear'; bf16 MFMA, f32 state; latent width L == 96).  Rows n:
 *   forward: x_0 = x0; a_j = relu(W1[:, :L] x_j + cvec[j]); x_{j+1} = x_j - (W2 a_j + b2)/S;
 *     v = W2 a_{S-1} + b2; nsx = x0 - v; d = Wst nsx + bst - zt; *loss += inv * sum d^2; dtr = 2 inv d;
 *     xS (optional) = x_{S-1} - v/S; X[j] = x_j and A[j] = a_j saved as bf16 (S, n, L) when non-NULL.
 *   backward: from dtr, the saved A and the optional gradient gxS of xS: DV[j] = dL/dv_j and
 *     DA[j] = dL/d(pre-activation of a_j) as bf16 (S, n, L), gx0 = dL/dx0 (f32).
 * W1 row stride ld_w1 (the time-embedding columns of meta_encoder.0 follow the first L). */
/* Fused relative-position attention backward (bf16 MFMA; NeMo RelPositionMultiHeadAttention,
 * Appendix A.7): from dO (rows, d), the forward's q+u / q+v rows, the fused q|k|v rows (ld 3d), the
 * projected positions pos (2T-1, d), the forward output O (rows, d) and the forward's per-row
 * log-sum-exp lse (B, H, T) with its bf16 unnormalised probabilities p_tilde (B, H, T, T) and per-64-key-block
 * running maxima m_blk (B, H, T, ceil(T/64)) (kdfm_relpos_attn_fwd), it forms P = p_tilde exp(m_blk - lse)
 * for dK / dV / dpos (DQ recomputes P = exp(S - lse) tile by tile and reads neither) and writes
 *   dqu = dS K, dqv_i = sum_j dS[i][j] pos[T-1-i+j]  (rows, d),  dK, dV into dqkv[:, d:] and [:, 2d:],
 *   dpos[r] = sum_{b,i} dS[i][r-T+1+i] qv_i  (2T-1, d, overwritten)
 * with dS = P (dP - r) scale, r_i = dO_i . O_i (= rowsum(dP P)) and dP the dropout-masked dO V^T (counter-RNG mask of the
 * forward).  The one T x T operand is the forward's bf16 p_tilde; deterministic (ordered chunk fold, no atomics).  Head
 * dim d/H <= 48.  ws: kdfm_relpos_attn_bwd_ws floats. */
int64_t kdfm_relpos_attn_bwd_ws(int64_t B, int64_t H, int64_t T, int64_t d);
/* The same backward issued in parts (a caller may put them on different streams): ROWDOT writes
 * D_i into ws; DQ, DKV and DPOS (+ its ordered fold) read it, so they must be ordered after ROWDOT
 * (same ws); DQ writes dqu / dqv, DKV dqkv[:, d:], DPOS dpos (the ws tail, which DQ / DKV do not touch). */
enum { KDFM_ATTN_BWD_ROWDOT = 1, KDFM_ATTN_BWD_DQ = 2, KDFM_ATTN_BWD_DKV = 4, KDFM_ATTN_BWD_DPOS = 8,
       KDFM_ATTN_BWD_ALL = 15 };
int kdfm_relpos_attn_bwd_parts(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                               const float* pos, const float* lse, const uint16_t* p_tilde, const float* m_blk,
                               const int64_t* lengths, float* dqu, float* dqv, float* dqkv, float* dpos, float* ws, int64_t ws_len, int64_t B, int64_t H, int64_t T,
                               int64_t d, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                               int32_t parts, void* stream);
int kdfm_relpos_attn_bwd(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                         const float* pos, const float* lse, const uint16_t* p_tilde, const float* m_blk,
                         const int64_t* lengths, float* dqu, float* dqv, float* dqkv, float* dpos,
                         float* ws, int64_t ws_len, int64_t B, int64_t H, int64_t T, int64_t d, float scale,
                         float dropout_p, const uint64_t* seed, uint64_t rng_stream, void* stream);
/* The backward in three kernels over SAVED probabilities (bwd2; the forward then writes only lse):
 *   _dq: r_i = dO_i . O_i formed in the dQ kernel's prologue (rsum: unused, may be NULL -- kept for the
 *        ABI), then dqu / dqv exactly as above (with the forward's key / value centring: dPd_ij =
 *        dO_i . (V_j - vc) + dO_i . vc, the second term in f32), and the bf16 score
 *        gradient dS and dropout-masked probabilities Pd = dropout(P) of every (i, j < len) written into
 *        ds / pd, each (B, H, T, ldt) with ldt = kdfm_relpos_attn_bwd2_ldt(T) (T rounded up to 8; keys
 *        >= len in the last written 64-key block are 0, key blocks past len and rows >= T unwritten);
 *   _dkv: dV[key] = sum_q Pd[q][key] dO_q, dK[key] = sum_q dS[q][key] qu_q into dqkv[:, 2d:] / [:, d:] --
 *        two plain products, no recompute of P, dP or the dropout mask;
 *   _dpos: dpos[r] = sum_{b,i} dS[i][r-T+1+i] qv_i (2T-1, d, overwritten) over per-utterance-chunk
 *        partials in ws (kdfm_relpos_attn_bwd2_dpos_ws floats) folded in chunk order.
 * _dkv and _dpos only read ds / pd: they may run concurrently on two streams after _dq.
 * Limits (32-bit buffer offsets): B*H*T*ldt*2 bytes of ds / pd and B*T*3d*4 bytes of qkv below 2 GiB
 * (KDFM_EINVAL otherwise). */
int64_t kdfm_relpos_attn_bwd2_ldt(int64_t T);
int64_t kdfm_relpos_attn_bwd2_dpos_ws(int64_t B, int64_t T, int64_t d);
int kdfm_relpos_attn_bwd2_dq(const float* dO, const float* O, const float* qu, const float* qv, const float* qkv,
                             const float* pos, const float* lse, const int64_t* lengths, float* rsum, uint16_t* ds,
                             uint16_t* pd, float* dqu, float* dqv, int64_t B, int64_t H, int64_t T, int64_t d,
                             float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream, void* stream);
int kdfm_relpos_attn_bwd2_dkv(const float* dO, const float* qu, const uint16_t* ds, const uint16_t* pd,
                              const int64_t* lengths, float* dqkv, int64_t B, int64_t H, int64_t T, int64_t d,
                              void* stream);
int kdfm_relpos_attn_bwd2_dpos(const float* qv, const uint16_t* ds, const int64_t* lengths, float* dpos, float* ws,
                               int64_t ws_len, int64_t B, int64_t H, int64_t T, int64_t d, void* stream);

/* Fused Conformer macaron feed-forward block (replaces the LayerNorm + Linear(d,ff)+SiLU+dropout +
 * Linear(ff,d)+dropout+residual of ConformerLayer.forward's feed_forward1 / feed_forward2 half steps,
 * NeMo conformer_modules.py, called conformer_encoder.py:685-692):
 *   out = x + rscale * drop_out(W2 drop_act(silu(W1 LN(x) + b1)) + b2)      (rows, d) fp32
 * bf16 MFMA, f32 state; the ff-wide hidden activation never reaches HBM.  Dropout masks use the
 * GEMM-epilogue flat indices (act: row*ff + n on stream_act, out: row*d + n on stream_out).
 * img: kdfm_ffn_img_elems(d, ff) bf16 prepared by kdfm_ffn_wprep from W1 (ff, d) / W2 (d, ff) fp32
 * (fwd_only: only the forward half of every chunk image is written).  mean / rstd (rows) fp32, or
 * both null (no backward).  Supported: d % 8 == 0 with d in (80, 96] or (160, 192], ff % 32 == 0
 * (kdfm_ffn_supported); all row operands 16-byte aligned.
 * Backward (dout = dL/dout): dx = dout + LN'(dln) with dln = W1^T dh, dh = (W2^T dl2) . drop_act' .
 * silu'(h), dl2 = rscale drop_out(dout); the hidden h is recomputed from LN(x).  Writes the bf16
 * weight-gradient operands ln_h (rows, d), a_h (rows, ff), dl2_h (rows, d), dh_h (rows, ff) for
 * kdfm_wgrad_bf16 (dW2 = dl2^T a, dW1 = dh^T ln) and the LayerNorm dgamma|dbeta partials `part` in
 * the kdfm_layernorm_bwd_part layout (kdfm_layernorm_bwd_ws(rows, d) floats) for kdfm_ln_fold. */
int32_t kdfm_ffn_supported(int64_t d, int64_t ff);

/* LayerNorm-fused input projections of the attention and convolution modules (ConformerLayer.forward,
 * SURVEY.md Appendix A.6/A.7; NeMo RelPositionMultiHeadAttention linear_q/k/v + pos_bias_u/v, and
 * ConformerConvolution pointwise_conv1 + GLU + pad mask; called conformer_encoder.py:685-692):
 *   kind 0 (QKV): ln = LN(x); [q|k|v] = ln W^T + bias (W (3d, d)); qu = q + pos_u, qv = q + pos_v (rows, d);
 *                 k, v into qkv[:, d:2d], qkv[:, 2d:3d] (rows, 3d; columns [0, d) are not written)
 *   kind 1 (GLU): ln = LN(x); [a|gate] = ln W^T + bias (W (2d, d)); g = a sigmoid(gate), 0 on frames
 *                 t >= lengths[b] (rows = B T, utterance-major)
 * bf16 MFMA, f32 state.  mean / rstd (rows) and ln_h (rows, d bf16, the weight-gradient operand) are
 * optional (null: not written).  img: kdfm_lnproj_img_elems(kind, d, bwd) bf16 from
 * kdfm_lnproj_wprep(kind, W, ...) (bwd = 0: forward image, 1: backward image).
 * Backward (d in (80, 96]): dx = dres + LN'(W^T dproj) with dproj = [dqu + dqv | dqkv[:, d:2d] |
 * dqkv[:, 2d:]] (QKV) or GLU'(dg) from the recomputed projection (GLU); writes ln_h, the bf16 dproj
 * (dqkv_h (rows, 3d) / da_h (rows, 2d): dW = dproj^T ln via kdfm_wgrad_bf16) and the LayerNorm
 * dgamma|dbeta partials `part` (kdfm_layernorm_bwd_part layout, folded by kdfm_ln_fold). */
int64_t kdfm_lnproj_img_elems(int32_t kind, int64_t d, int32_t bwd);

/* Row-streaming d x d products of a Conformer layer (attention linear_out, conv pointwise_conv2 and
 * their data gradients; ConformerLayer.forward, SURVEY.md Appendix A.6/A.7, called
 * conformer_encoder.py:685-692): out = epi(pro(x) Wop^T) over (rows, d) fp32 rows, bf16 MFMA.
 *   prologue 0: x;  1 (dropout): x * s_in * keep(row*d + k, stream_in) / (1 - p_in);
 *            2 (BN-SiLU): silu((x - bn_mean) bn_rstd bn_g + bn_b) per channel
 *   x_h (optional, rows x d bf16): the prologue output as the weight-gradient operand
 *   epilogue 0: acc;  1 (residual): R + rscale * drop(acc + bias) (mask row*d + n on stream_out)
 * img: kdfm_rowgemm_img_elems(d) bf16 from kdfm_rowgemm_wprep(W (d, d) [out][in]; trans = 1 for the
 * data gradient dx = dy W).  d as kdfm_ffn_supported; rows 16-byte aligned. */
int64_t kdfm_rowgemm_img_elems(int64_t d);

/* Every weight image of a model in ONE launch per step: a device array of jobs (the host builds it
 * once; pointers stay valid while the parameter buffer lives), each job one image of the fused
 * Conformer kernels above.  start = first global thread of the job (jobs in increasing start, each
 * kdfm_wimg_job_threads(job) threads); total_threads = sum over jobs. */
typedef struct kdfm_wimg_job {
  int64_t type;   /* 0: FFN chunk image (W1, W2; kdfm_ffn_wprep), 1: LN projection (W1 = W;
                     kdfm_lnproj_wprep), 2: row-streaming (W1 = W; kdfm_rowgemm_wprep) */
  int64_t kind;   /* LN projection: 0 QKV, 1 GLU */
  int64_t flag;   /* FFN: forward-only image; LN projection: backward image; row-streaming: transposed */
  int64_t d, ff;
  const float* W1;
  const float* W2;
  uint16_t* img;
  int64_t start;
} kdfm_wimg_job;
int64_t kdfm_wimg_job_threads(const kdfm_wimg_job* job);
int kdfm_wimg_prep_batch(const kdfm_wimg_job* jobs, int32_t njobs, int64_t total_threads, void* stream);
int kdfm_rowgemm_wprep(const float* W, uint16_t* img, int64_t d, int32_t trans, void* stream);
int kdfm_rowgemm(const float* x, const uint16_t* img, float* out, int64_t rows, int64_t d, int32_t prologue,
                 float p_in, float s_in, uint64_t stream_in, const float* bn_mean, const float* bn_rstd,
                 const float* bn_g, const float* bn_b, uint16_t* x_h, int32_t epilogue, const float* bias,
                 const float* R, float rscale, float p_out, uint64_t stream_out, const uint64_t* seed,
                 void* stream);
int kdfm_lnproj_wprep(int32_t kind, const float* W, uint16_t* img, int64_t d, int32_t bwd, void* stream);
int kdfm_ln_qkv_fwd(const float* x, const float* ln_g, const float* ln_b, float ln_eps, const uint16_t* img,
                    const float* bias, const float* pos_u, const float* pos_v, float* qu, float* qv, float* qkv,
                    float* mean, float* rstd, uint16_t* ln_h, int64_t rows, int64_t d, void* stream);
int kdfm_ln_glu_fwd(const float* x, const float* ln_g, const float* ln_b, float ln_eps, const uint16_t* img,
                    const float* bias, const int64_t* lengths, int64_t T, float* g, float* mean, float* rstd,
                    uint16_t* ln_h, int64_t rows, int64_t d, void* stream);
/* part_uv (optional, kdfm_layernorm_bwd_ws(rows, d) floats): the pos_bias_u | pos_bias_v gradients
 * (column sums of dqu | dqv) as 16-row-group partials in the same layout, folded by kdfm_ln_fold. */
int kdfm_ln_qkv_bwd(const float* dqu, const float* dqv, const float* dqkv, const float* x, const float* mean,
                    const float* rstd, const float* ln_g, const float* ln_b, const uint16_t* img, const float* dres,
                    float* dx, uint16_t* ln_h, uint16_t* dqkv_h, float* part, float* part_uv, int64_t rows, int64_t d,
                    void* stream);
int kdfm_ln_glu_bwd(const float* dg, const float* x, const float* mean, const float* rstd, const float* ln_g,
                    const float* ln_b, const uint16_t* img, const float* bias, const int64_t* lengths, int64_t T,
                    const float* dres, float* dx, uint16_t* ln_h, uint16_t* da_h, float* part, int64_t rows,
                    int64_t d, void* stream);
int64_t kdfm_ffn_img_elems(int64_t d, int64_t ff);
int kdfm_ffn_wprep(const float* W1, const float* W2, uint16_t* img, int64_t d, int64_t ff, int32_t fwd_only,
                   void* stream);
/* out_ln (optional): the layer's norm_out fused into the epilogue, out_ln = LN(out; out_ln_g, out_ln_b,
 * out_ln_eps) with its row statistics in out_ln_mean / out_ln_rstd (all null: not computed). */
int kdfm_ffn_fwd(const float* x, const float* ln_g, const float* ln_b, float ln_eps, const uint16_t* img,
                 const float* b1, const float* b2, float* out, float* mean, float* rstd, int64_t rows, int64_t d,
                 int64_t ff, float rscale, float p_act, float p_out, const uint64_t* seed, uint64_t stream_act,
                 uint64_t stream_out, const float* out_ln_g, const float* out_ln_b, float out_ln_eps, float* out_ln,
                 float* out_ln_mean, float* out_ln_rstd, void* stream);
int kdfm_ffn_bwd(const float* dout, const float* x, const float* mean, const float* rstd, const float* ln_g,
                 const float* ln_b, const uint16_t* img, const float* b1, float* dx, uint16_t* ln_h, uint16_t* a_h,
                 uint16_t* dl2_h, uint16_t* dh_h, float* part, int64_t rows, int64_t d, int64_t ff, float rscale,
                 float p_act, float p_out, const uint64_t* seed, uint64_t stream_act, uint64_t stream_out,
                 void* stream);

int kdfm_fm_chain_fwd(const float* x0, const float* zt, const float* W1, int64_t ld_w1, const float* cvec,
                      const float* W2, const float* b2, const float* Wst, const float* bst, uint16_t* X, uint16_t* A,
                      float* nsx, float* dtr, float* xS, float* loss, float inv, int64_t n, int32_t L, int32_t S,
                      void* stream);
int kdfm_fm_chain_bwd(const float* dtr, const uint16_t* A, const float* gxS, const float* W1, int64_t ld_w1,
                      const float* W2, const float* Wst, uint16_t* DV, uint16_t* DA, float* gx0, int64_t n, int32_t L,
                      int32_t S, void* stream);
/* Encoder-level flow matching with the dynamic step router (asr_train.py DistilFlowMatchingCTCModelBPE,
 * use_flow_matching + use_dynamic_steps; DynamicStepRouter :1021-1218, FlowMatchingModule :1220-1377 with
 * meta_encoder 'mlp' [Cs+32 -> 128 -> Cs], time_embed Linear(1, 32), shape_transform Linear(Cs, Ct), MSE; the
 * per-layer loop of forward() :595-666).  All L hooked layers at once: rows are (layer, utterance, frame)
 * = segment u = l*B + b of T frames, features (L*B*T, Cs) student / (L*B*T, Ct) teacher.
 *   kdfm_encfm_time_prep:  c01 = [c0 | c1] (2 x 128): c0 = b1 + W1e b_te, c1 = W1e w_te (time bias c0 + t c1)
 *   kdfm_encfm_router_fwd: per segment: time means sv, tv; hcat = [relu(Wsp sv + bsp) | relu(Wtp tv + btp) |
 *     emb[l]] (288); h0 = relu(W0 hcat + b0) (128); logits = W2 h0 + b2 (K); probs = softmax (min_steps mask);
 *     ent = -sum p log max(p, 1e-8); steps = argmax(logits + g) + 1 with g Gumbel(0,1) (the `gumbel` (U, K)
 *     array, else counter RNG (seed, rng_stream)) when train, argmax(logits) + 1 otherwise
 *   kdfm_encfm_strategy: per layer the flow step counts S[u] (0 batch_mode: smallest most frequent;
 *     1 batch_avg: round-half-even of the mean, clamped to [1, K]; 2 batch_median: lower median; 3 group:
 *     S[u] = steps[u]), the MSE weights inv[u] = 1 / (elements of the FM call the segment belongs to), the
 *     compact save offsets off[u] = T * sum_{v<u} S[v] and rows_total = T * sum S; the router loss
 *     rloss[l] = budget_weight (mean steps - budget_target)^2 - entropy_weight mean ent (train) and mean_steps[l]
 *   kdfm_encfm_chain_fwd: per row (S = S[u]): x_0 = x0; for j < S, t = (S - j) / S:
 *     a_j = relu(W1x x_j + c0 + t c1); v_j = W2 a_j + b2; x_{j+1} = x_j - v_j / S;
 *     nsx = ca[S] x0 + cv[S] v_{S-1} (noise_scheduled_x at t = 1/S: (dalpha s - v) / (-dsigma));
 *     d = Wst nsx + bst - tf; loss[l] += inv[u] sum d^2; dtr = 2 inv[u] d; rows >= xs_row0: xS = x_S;
 *     saves (bf16, compact rows off[u] + j T + frame): X = [x_j | 1 | t | 0] (96 wide), A = a_j (128)
 *   kdfm_encfm_chain_bwd: the data gradients: dnsx = Wst^T dtr; g = gxS (rows >= xs_row0) or 0;
 *     j = S-1..0: dv_j = (j == S-1 ? cv dnsx : 0) - g / S; da_j = (W2^T dv_j) . [a_j > 0]; g += W1x^T da_j;
 *     gx0 = g + ca dnsx + dsv[u] / T (the router's time-mean gradient, optional); saves DV (Cs), DA (128)
 *     Weight gradients: kdfm_wgrad_bf16_dev(DA, X -> W1[:, :96] (dW1x | dc0 | dc1), rows_total) and
 *     (DV, A -> W2, b2), the f32 row-parallel gradient of (dtr, nsx -> Wst, bst), then kdfm_encfm_time_bwd.
 *   kdfm_encfm_router_bwd: dlogits = coef dH/dlogits (coef = -router_weight entropy_weight / B; the budget
 *     term has no gradient), dh0 = W2^T dlogits . [h0 > 0], dhcat = W0^T dh0 (ReLU masks on the projections),
 *     dsv = Wsp^T dhcat[:128]; weight gradients by the caller ((dlogits, h0), (dh0, hcat), (dhcat[:128], sv),
 *     (dhcat[128:256], tv))
 *   kdfm_encfm_time_bwd: from dW1's columns Cs (dc0) and Cs+1 (dc1): gb1 += dc0; gW1[:, Cs:] = dc0 b_te^T +
 *     dc1 w_te^T (overwritten); gw_te += W1e^T dc1; gb_te += W1e^T dc0; gemb[l] += sum_b dhcat[u][256:288].
 * Hidden widths fixed at 128 (FM and router), time / layer embeddings 32; Cs + 2 <= 96, Ct <= 192, steps <= 16.
 * ca / cv: host arrays of the schedule coefficients for S = 1..max_steps. */
int kdfm_encfm_time_prep(const float* W1, int64_t ld_w1, const float* b1, const float* w_te, const float* b_te,
                         int32_t Cs, int32_t H, int32_t E, float* c01, void* stream);
int kdfm_encfm_router_fwd(const float* s, const float* t, const float* Wsp, const float* bsp, const float* Wtp,
                          const float* btp, const float* emb, const float* W0, const float* b0, const float* W2,
                          const float* b2, const float* gumbel, const uint64_t* seed, uint64_t rng_stream,
                          int32_t train, float* sv, float* tv, float* hcat, float* h0, float* probs, float* ent,
                          int32_t* steps, int64_t L, int64_t B, int64_t T, int32_t Cs, int32_t Ct, int32_t K,
                          int32_t P, int32_t E, int32_t min_steps, void* stream);
int kdfm_encfm_strategy(const int32_t* steps, const float* ent, int32_t* S, float* inv, int64_t* off,
                        int64_t* rows_total, float* rloss, float* mean_steps, int64_t L, int64_t B, int64_t T,
                        int32_t K, int32_t Ct, int32_t strategy, float budget_target, float budget_weight,
                        float entropy_weight, int32_t train, void* stream);
int kdfm_encfm_chain_fwd(const float* x0, const float* tf, const int32_t* S, const float* inv, const int64_t* off,
                         const float* W1, int64_t ld_w1, const float* c01, const float* W2, const float* b2,
                         const float* Wst, const float* bst, const float* ca, const float* cv, int32_t max_steps,
                         uint16_t* X, uint16_t* A, float* nsx, float* dtr, float* xS, int64_t xs_row0, float* loss,
                         int64_t L, int64_t B, int64_t T, int32_t Cs, int32_t Ct, void* stream);
int kdfm_encfm_chain_bwd(const float* dtr, const uint16_t* A, const float* gxS, int64_t xs_row0, const int32_t* S,
                         const int64_t* off, const float* W1, int64_t ld_w1, const float* W2, const float* Wst,
                         const float* ca, const float* cv, int32_t max_steps, const float* dsv, uint16_t* DV,
                         uint16_t* DA, float* gx0, int64_t L, int64_t B, int64_t T, int32_t Cs, int32_t Ct,
                         void* stream);
int kdfm_encfm_router_bwd(const float* probs, const float* hcat, const float* h0, const float* W2, const float* W0,
                          const float* Wsp, float coef, float* dlogits, float* dh0, float* dhcat, float* dsv,
                          int64_t L, int64_t B, int32_t Cs, int32_t K, void* stream);
int kdfm_encfm_time_bwd(float* gW1, int64_t ld_w1, float* gb1, const float* W1, const float* w_te, const float* b_te,
                        float* gw_te, float* gb_te, const float* dhcat, float* gemb, int64_t L, int64_t B, int32_t Cs,
                        void* stream);
/* Fused SimpleDenoiser chain (asr_train_diffm.py:444-460: S steps of x <- x - net(x)/S, net =
 * Conv1d(L,L,3,p=1) -> ReLU -> Conv1d(L,L,3,p=1); bf16 MFMA, f32 state; L == 96) over n rows =
 * (n / T) utterances of T frames, channels-last.  W1 / W2: PyTorch Conv1d weights (L, L, 3) fp32.
 *   forward:  out = x_S;  saves X[i] = x_i and A[i] = relu(conv1(x_i) + b1) as bf16 (S, n, L)
 *   backward: gout = dL/dx_S -> gin = dL/dx_0;  saves GV[i] = dL/dx_{i+1} and
 *             DA[i] = -(1/S) conv2^T(GV[i]) . [A[i] > 0] as bf16 (S, n, L)
 * Weight gradients: kdfm_wgrad_bf16_conv(DA, X) and (GV, A) with alpha -1/S over S n rows. */
int64_t kdfm_denoise_wimg_elems(void);   /* bf16 elements of the wimg workspace (prepared weight images) */
int kdfm_denoise_chain_fwd(const float* z, const float* W1, const float* b1, const float* W2, const float* b2,
                           uint16_t* wimg, uint16_t* X, uint16_t* A, float* out, int64_t n, int64_t T, int32_t L,
                           int32_t S, void* stream);
int kdfm_denoise_chain_bwd(const float* gout, const uint16_t* A, const float* W1, const float* W2, uint16_t* wimg,
                           uint16_t* GV, uint16_t* DA, float* gin, int64_t n, int64_t T, int32_t L, int32_t S,
                           void* stream);
/* bf16 weight twins (once per step, before the GEMMs that read them):
 *   kdfm_cast_bf16:   dst[i] = bf16(src[i]), i < n  (same layout as the f32 flat parameter buffer)
 *   kdfm_cast_bf16_t: per table entry e = (offset, rows, cols, first_block) (device int64 [ntab][4]):
 *     dst[offset + c*rows + r] = bf16(src[offset + r*cols + c]) — each 2-D weight transposed in
 *     place of itself; first_block = prefix sum of ceil(rows*cols/256); nblocks = total. */
int kdfm_cast_bf16(const float* src, uint16_t* dst, int64_t n, void* stream);
int kdfm_cast_bf16_t(const float* src, uint16_t* dst, const int64_t* table, int64_t ntab, int64_t nblocks,
                     void* stream);
int64_t kdfm_gemm_ws(const kdfm_gemm_desc* d); /* workspace elements kdfm_gemm would use (0: none) */
/* kernel family the calling thread's most recent kdfm_gemm launched (profiling attribution):
 * 0 generic 64x64 MFMA tile, 1 weight-stationary skinny, 2 row-streaming forward, 3 wide-tile
 * weight gradient + fold, 4 generic tile with ordered split-K fold, 5 LDS-slab k=3 conv,
 * 6 row-parallel weight gradient + ordered fold; -1 none */
int32_t kdfm_gemm_last_route(void);

/* column sums: out[n] (+)= scale * sum_m X[m*ld + n], m < M; accumulate != 0 adds into out.
 * (bias gradients of every Linear / Conv1d on the path) */
int kdfm_colsum(const float* X, float* out, int64_t M, int64_t N, int64_t ld, float scale, int32_t accumulate,
                void* stream);

/* ---------------- frontend: AudioToMelSpectrogramPreprocessor (audio_preprocessing.py:214-300,
 * FilterbankFeatures semantics SURVEY Appendix A.1) --------------------------------------- */
/* xp (B, N + 2*pad): zero-centre-padded preemphasised signal, masked beyond lengths[b];
 * optional dither (training) from the counter RNG. */
int kdfm_preemph_pad(const float* wav, const int64_t* lengths, float* xp, int64_t B, int64_t N, int64_t pad,
                     float preemph, float dither, const uint64_t* seed, uint64_t rng_stream, void* stream);
/* power[r, f] = spec[r, f]^2 + spec[r, nbins + f]^2 (spec rows = [re | im] from the DFT GEMM) */
int kdfm_power_spectrum(const float* spec, float* power, int64_t rows, int64_t nbins, void* stream);
/* Mel power spectrum via a 512-point real FFT per frame (FilterbankFeatures, audio_preprocessing.py:
 * 93-103, 214-300): mel[f][m] = sum_{k in [fb_lo[m], fb_hi[m])} fb[m][k] |X_f[k]|^2 with
 * X_f = FFT_512(window (win taps, centred) * xp[b][t hop + n]), f = b T + t; twiddle = e^{-2 pi i j/512}
 * as (re, im) float pairs, j < 512; fb (nfilt, 257) row-major.  Replaces the DFT-as-GEMM + power +
 * filterbank GEMM chain (same arithmetic in f32, ~35x fewer flops). */
int kdfm_logmel_fft(const float* xp, int64_t ldx, const float* window, const float* twiddle, const float* fb,
                    const int32_t* fb_lo, const int32_t* fb_hi, float* mel, int64_t B, int64_t T, int64_t hop,
                    int64_t n_fft, int64_t win, int64_t nfilt, void* stream);
/* log(mel + guard), per-feature mean / unbiased std over valid frames, zero beyond seq_len;
 * mel/out laid out (B, T, nfilt). */
int kdfm_logmel_normalize(const float* mel, const int64_t* seq_len, float* out, int64_t B, int64_t T, int64_t nfilt,
                          float log_guard, void* stream);
/* SpectrogramAugmentation (audio_preprocessing.py:443-553, called asr_train_diffm.py:622-623; NeMo's
 * vectorized SpecAugment, the use_vectorized_spec_augment=True default), in place on
 * (B, T, nfilt): per utterance, time mask q has width (int)(U * min(time_width * len, T)) and start
 * (int)(U' * (len - width)); frequency mask q width (int)(U * freq_width), start (int)(U' * (nfilt - width));
 * f32 arithmetic.  uniforms (optional, B x 2 (time_masks + freq_masks) floats in [0, 1), per utterance
 * [time widths | time starts | freq widths | freq starts]): the draws as an input (parity mode); NULL =
 * drawn from the counter RNG (seed, rng_stream).  mask_out (optional, uint8) records the masked cells. */
int kdfm_specaugment(float* x, const int64_t* seq_len, uint8_t* mask_out, int64_t B, int64_t T, int64_t nfilt,
                     int32_t freq_masks, int32_t freq_width, int32_t time_masks, float time_width,
                     const uint64_t* seed, uint64_t rng_stream, const float* uniforms, void* stream);

/* ---------------- ConvSubsampling 'striding' (conformer_encoder.py:381-390, 635; A.3) ------- */
/* cols[(b,t2,f2), c*9 + ky*3 + kx] = X[b, 2t2-1+ky, 2f2-1+kx, c] ; X channels-last (B,T1,F1,C),
 * frames >= len_in[b] read as zero (padding mask). */
int kdfm_im2col_3x3s2(const float* X, const int64_t* len_in, float* cols, int64_t B, int64_t T1, int64_t F1,
                      int64_t C, void* stream);
/* Striding subsampling forward in one kernel (bf16 MFMA; conformer_encoder.py:381-390, 635; A.3):
 * y2 = mask2(ReLU(conv2(mask1(ReLU(conv1(mask0(mel))))))) with conv1 / conv2 = Conv2d(3x3, stride 2,
 * pad 1), mel (B, Tm, F = 80) f32, y2 (B * T2 * 20, C) f32 channels-last rows; conv1 is computed on the
 * fly per workgroup (MFMA over hi/lo bf16 splits of the mel taps and weights, f32 accumulation) and never
 * leaves LDS, except that y1 (optional, (B * T1 * 40, ldy1) bf16) receives the conv1 output for a trained
 * student's backward: ldy1 a multiple of 8 in [C, 32 ceil(C / 32)], channels [C, ldy1) written as zeros (96 at
 * C = 88: whole 64-byte row segments per 32-channel chunk).  y1, y2, wp 16-byte aligned.  mel_len / len1 / len2 (optional): the frame masks.  wp: kdfm_subsample_fused_wprep's
 * operand image of (w0 (C,1,3,3), w2 (C,C,3,3)), kdfm_subsample_fused_wprep_elems(C) bf16.
 * C in {88, 96, 176, 192} (kdfm_subsample_fused_supported). */
int kdfm_subsample_fused_supported(int64_t C, int64_t F);
int64_t kdfm_subsample_fused_wprep_elems(int64_t C);
int kdfm_subsample_fused_wprep(const float* w0, const float* w2, uint16_t* wp, int64_t C, void* stream);
int kdfm_subsample_fused(const float* mel, const int64_t* mel_len, const int64_t* len1, const int64_t* len2,
                         const uint16_t* wp, const float* b0, const float* b2, float* y2, uint16_t* y1, int64_t B,
                         int64_t Tm, int64_t F, int64_t C, int64_t ldy1, void* stream);
/* Tap-major bf16 columns: cols[(b,t2,f2), tap*C + c] = bf16(X[b, 2 t2 - 1 + ky, 2 f2 - 1 + kx, c]) (0 outside /
 * beyond len_in), C % 8 == 0; the bf16 step's conv2 weight-gradient operand. */
/* the same tap-major bf16 columns from a bf16 source (the saved bf16 conv1 output y1) */
int kdfm_im2col_3x3s2_tm_from_bf16(const uint16_t* X, const int64_t* len_in, uint16_t* cols, int64_t B, int64_t T1,
                                   int64_t F1, int64_t C, void* stream);
int kdfm_im2col_3x3s2_tm_bf16(const float* X, const int64_t* len_in, uint16_t* cols, int64_t B, int64_t T1, int64_t F1,
                              int64_t C, void* stream);
/* adjoint of the above (gather form); optionally multiplied by relu'(relu_out). */
int kdfm_col2im_3x3s2(const float* dcols, const int64_t* len_in, const float* relu_out, float* dX, int64_t B,
                      int64_t T1, int64_t F1, int64_t C, void* stream);
/* the same adjoint for a tap-major dcols (column tap*C + c, tap = ky*3 + kx): produced by the
 * data-gradient GEMM against the (C, 9, C) re-laid weight, read with contiguous lanes */
int kdfm_col2im_3x3s2_tapmajor(const float* dcols, const int64_t* len_in, const float* relu_out, float* dX, int64_t B,
                      int64_t T1, int64_t F1, int64_t C, void* stream);

/* ---------------- ConvSubsampling 'dw_striding' (conformer_encoder.py:381-390; recipe
 * fast-conformer_ctc_bpe.yaml:122-125): Conv2d(1->C,3,s2)+ReLU, then per further stage a depthwise
 * Conv2d(C,3,s2,groups=C) + pointwise 1x1 (kdfm_gemm, EPI_BIAS|RELU|ROWMASK) + ReLU; NeMo's masked
 * conv sequence zeroes frames >= each layer's length before and after it.  Activations
 * channels-last (B, T, F, C), C % 4 == 0, 16-byte aligned; weights (C, 1, 3, 3), bias (C).
 * Padding (pad_t, pad_f) = left padding of both axes (1 symmetric, 2 for CausalConv2D). */
/* out[i] = floor((in[i] + pad_total - kernel) / stride) + 1 (NeMo calc_length, one stage) */
int kdfm_conv_lengths(const int64_t* in, int64_t* out, int64_t n, int32_t pad_total, int32_t kernel, int32_t stride,
                      void* stream);
/* y[b,to,fo,c] = mask(to < out_len[b]) * act(bias[c] + sum_{i,j} w[c,i,j] * x[b, 2to-pad_t+i, 2fo-pad_f+j, Cin==1 ? 0 : c])
 * with x frames >= in_len[b] (and outside the input) read as zero; act = relu when relu != 0.
 * in_len / out_len may be NULL (no mask). */
int kdfm_dwsub_conv(const float* x, const int64_t* in_len, const float* w, const float* bias, float* y,
                    const int64_t* out_len, int64_t B, int64_t Ti, int64_t Fi, int64_t Cin, int64_t C, int64_t To,
                    int64_t Fo, int32_t pad_t, int32_t pad_f, int32_t relu, void* stream);
/* data gradient of the depthwise layer (Cin == C): dx = adjoint(dy masked at out_len), times
 * relu'(x_saved) when x_saved != NULL (the layer's input was a ReLU output), zero at ti >= in_len. */
int kdfm_dwsub_conv_dgrad(const float* dy, const int64_t* out_len, const float* w, const float* x_saved,
                          const int64_t* in_len, float* dx, int64_t B, int64_t Ti, int64_t Fi, int64_t C, int64_t To,
                          int64_t Fo, int32_t pad_t, int32_t pad_f, void* stream);
/* weight and bias gradients dw (C,1,3,3), db (C) of kdfm_dwsub_conv (Cin 1 or C): per-slab partials
 * in ws then an ordered fold (deterministic in every mode); accumulate != 0 adds into dw/db.
 * kdfm_dwsub_conv_wgrad_ws gives the workspace size in floats. */
int64_t kdfm_dwsub_conv_wgrad_ws(int64_t B, int64_t To, int64_t Fo, int64_t C);
int kdfm_dwsub_conv_wgrad(const float* dy, const int64_t* out_len, const float* x, const int64_t* in_len, float* dw,
                          float* db, float* ws, int64_t ws_len, int64_t B, int64_t Ti, int64_t Fi, int64_t Cin,
                          int64_t C, int64_t To, int64_t Fo, int32_t pad_t, int32_t pad_f, int32_t accumulate,
                          void* stream);

/* Fused striding subsampling forward (bf16 MFMA mode; replaces im2col + GEMM for the same A.3
 * arithmetic, conformer_encoder.py:381-390, 635):
 *   kdfm_subsample_conv1: y1[(b,t1,f1), c] = mask(t1 < len1[b]) * relu(b0[c] + sum_tap w0[c,tap] *
 *     mel[b, 2t1-1+ky, 2f1-1+kx]) with mel frames >= mel_len[b] read as zero; mel channels-last
 *     (B,Tm,F); y1b bf16 (B,T1,F1,C) and optionally y1f f32 (same layout).  C % 8 == 0.
 *   kdfm_subsample_wprep: conv2 weight (C,C,3,3) f32 -> bf16 image [Np][9][Cp] (Np = C rounded up
 *     to 32, Cp = C rounded up to 16, zero padded); kdfm_subsample_wprep_elems gives its size.
 *   kdfm_subsample_conv2: implicit GEMM y2[(b,t2,f2), c] = mask(t2 < len2[b]) * relu(b2[c] +
 *     sum_{tap,ci} W2[c,ci,tap] y1[b, 2t2-1+ky, 2f2-1+kx, ci]); y2 f32 channels-last.  C <= 192. */
int64_t kdfm_subsample_wprep_elems(int64_t C);
int kdfm_subsample_wprep(const float* w2, uint16_t* wb, int64_t C, void* stream);
int kdfm_subsample_conv1(const float* mel, const int64_t* mel_len, const int64_t* len1, const float* w0,
                         const float* b0, uint16_t* y1b, float* y1f, int64_t B, int64_t Tm, int64_t F, int64_t C,
                         void* stream);
int kdfm_subsample_conv2(const uint16_t* y1b, const int64_t* len2, const uint16_t* wb, const float* b2, float* y2,
                         int64_t B, int64_t T1, int64_t F1, int64_t C, void* stream);
/* conv2's data gradient without an im2col matrix (bf16 MFMA, f32 accumulate):
 *   dy1[b,t1,f1,ci] = [y1 > 0] * sum_{ky,kx,co: 2 t2 - 1 + ky = t1, 2 f2 - 1 + kx = f1} W[co,ci,ky,kx] dy2[b,t2,f2,co]
 * over the parity classes of (t1, f1) (1, 2, 2 or 4 taps each); wt = kdfm_subsample_dgrad_wprep(W)
 * (kdfm_subsample_dgrad_wprep_elems(C) bf16); y1 = the bf16 conv1 output (only its sign is read).
 * Replaces the ConvSubsampling backward's linear_dx into
 * (B T2 F2, 9C) columns + col2im (conformer_encoder.py:381-390). */
int64_t kdfm_subsample_dgrad_wprep_elems(int64_t C);
int kdfm_subsample_dgrad_wprep(const float* w2, uint16_t* wt, int64_t C, void* stream);
/* The same data gradient with ConvSubsampling conv0's weight gradient fused into its epilogue (the
 * striding path: conv0 = Conv2d(1 -> C, 3x3, stride 2, pad) over the (B, Tm, Fm) mel frames, frames
 * t >= mel_len[b] read as zero; mel_len may be null): dw0 (C, 9) += sum dy1 x_patch, db0 (C) += sum dy1,
 * from per-workgroup partials in ws (kdfm_subsample_conv2_dgrad_w0_ws floats) folded in workgroup order.
 * dy1 may be null (not written).  Requires B T1 F1 < 2^24.  ldy1 (>= C): y1's row stride in elements (the fused
 * forward's padded rows); dy1 is (B T1 F1, C). */
int64_t kdfm_subsample_conv2_dgrad_w0_ws(int64_t B, int64_t T1, int64_t F1, int64_t C);
int kdfm_subsample_conv2_dgrad_w0(const float* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B,
                                  int64_t T1, int64_t F1, int64_t C, int64_t ldy1, const float* mel,
                                  const int64_t* mel_len, int64_t Tm, int64_t Fm, int64_t pad, float* dw0, float* db0,
                                  float* ws, int64_t ws_len, void* stream);
int kdfm_subsample_conv2_dgrad(const float* dy2, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B, int64_t T1,
                               int64_t F1, int64_t C, int64_t ldy1, void* stream);
/* The same with a bf16 dy2 (kdfm_ss_out_dgrad's output): one 16-byte load of 8 channels per k-step instead of
 * two f32 ones (the tap re-reads of dy2 are the kernel's dominant traffic). */
int kdfm_subsample_conv2_dgrad_w0_h(const uint16_t* dy2h, const uint16_t* wt, const uint16_t* y1, float* dy1, int64_t B,
                                    int64_t T1, int64_t F1, int64_t C, int64_t ldy1, const float* mel,
                                    const int64_t* mel_len, int64_t Tm, int64_t Fm, int64_t pad, float* dw0, float* db0,
                                    float* ws, int64_t ws_len, void* stream);
/* Subsampling output Linear(C F2 -> d) backward into the conv2 output gradient (replaces linear_dx with the
 * DRELU epilogue + a bf16 cast; conformer_encoder.py:381-390 ConvSubsampling.out): with the channels-last
 * conv2 output y2 (rows, ncols = F2 C) f32 and dlin (rows, d) f32,
 *   dy2h[r][n] = bf16([y2[r][n] > 0] * sum_{k < d} bf16(dlin[r][k]) bf16(W[k][n]))   (f32 accumulation).
 * kdfm_ss_out_wprep writes wt = W^T as bf16 [ncols][32 ceil(d / 32)] (kdfm_ss_out_wprep_elems elements; W is
 * the (d, ncols) re-laid output weight).  d <= 128, ncols % 4 == 0. */
int64_t kdfm_ss_out_wprep_elems(int64_t d, int64_t ncols);
int kdfm_ss_out_wprep(const float* W, uint16_t* wt, int64_t d, int64_t ncols, void* stream);
int kdfm_ss_out_dgrad(const float* dlin, const uint16_t* wt, const float* y2, uint16_t* dy2h, int64_t rows, int64_t d,
                      int64_t ncols, void* stream);

/* ---------------- Evaluation path (ctc_models.py:625-692, wer.py) ---------
 * kdfm_ctc_greedy: CTC greedy decoding (Appendix A.9; WER.update wer.py:329-333): per utterance b,
 *   argmax over C classes of frames t < lengths[b] (first index on ties), collapse repeats when
 *   fold != 0, drop `blank`; tokens[b*T + i], i < ntok[b] (int32); optional labels[b*T + t] = the
 *   per-frame argmax (blank beyond the length).  log_probs rows (b*T + t) with row stride ld.
 * kdfm_edit_distance: host-side Levenshtein distance between two int32 sequences (editdistance.eval,
 *   wer.py:66-69); -1 on bad arguments.  No device work. */
int kdfm_ctc_greedy(const float* log_probs, int64_t ld, const int64_t* lengths, int32_t* tokens, int32_t* ntok,
                    int32_t* labels, int64_t B, int64_t T, int64_t C, int64_t blank, int32_t fold, void* stream);
int64_t kdfm_edit_distance(const int32_t* a, int64_t na, const int32_t* b, int64_t nb);

/* ---------------- ConformerLayer (Appendix A.5-A.8; layers built conformer_encoder.py:450-472) */
int kdfm_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd,
                       int64_t rows, int64_t d, float eps, void* stream);
/* The same LayerNorm with a bf16 y (round to nearest even) for an LN output whose every consumer reads bf16 operands
 * (the large-tile GEMM's forward and weight gradient, FastConformer(-XL)); d % 256 == 0, 16-byte aligned rows. */
int kdfm_layernorm_fwd_bf16(const float* x, const float* gamma, const float* beta, uint16_t* y, float* mean,
                            float* rstd, int64_t rows, int64_t d, float eps, void* stream);
/* dx = LN'(dy) (+ dres if non-null); dgamma/dbeta accumulate (+=). */
/* dgamma/dbeta are accumulated (+=) through per-block partials in ws, which must hold at least
 * kdfm_layernorm_bwd_ws(rows, d) floats (no zeroing needed) */
int kdfm_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                       const float* dres, float* dx, float* dgamma, float* dbeta, float* ws, int64_t rows, int64_t d,
                       void* stream);
int64_t kdfm_layernorm_bwd_ws(int64_t rows, int64_t d);
/* the same backward with the fold deferred: dgamma|dbeta block partials are written to `part`
 * (kdfm_layernorm_bwd_ws(rows, d) floats) and folded later, for up to KDFM_LN_FOLD_MAX LayerNorms of
 * the same (rows, d) in one launch, by kdfm_ln_fold (dgamma[i] / dbeta[i] accumulate, block order:
 * deterministic).  parts / dgamma / dbeta are HOST arrays of n device pointers. */
#define KDFM_LN_FOLD_MAX 8
int kdfm_layernorm_bwd_part(const float* dy, const float* x, const float* gamma, const float* mean,
                            const float* rstd, const float* dres, float* dx, float* part, int64_t rows, int64_t d,
                            void* stream);
/* the same with dy + dy2 as the output gradient (summed on load: the encoder backward's layer-input
 * gradient plus the next hooked output's, without an add launch) */
int kdfm_layernorm_bwd_part2(const float* dy, const float* dy2, const float* x, const float* gamma, const float* mean,
                             const float* rstd, const float* dres, float* dx, float* part, int64_t rows, int64_t d,
                             void* stream);
int kdfm_ln_fold(const float* const* parts, float* const* dgamma, float* const* dbeta, int32_t n, int64_t rows,
                 int64_t d, void* stream);
/* Qu = Q + pos_bias_u, Qv = Q + pos_bias_v from the fused (rows, 3d) q|k|v projection */
int kdfm_qkv_prep(const float* qkv, const float* pos_bias_u, const float* pos_bias_v, float* qu, float* qv,
                  int64_t rows, int64_t d, void* stream);
/* softmax((AC + rel_shift(BD)) * scale) with NeMo masking, optional dropout_att -> Pdrop */
int kdfm_relpos_softmax_fwd(const float* ac, const float* bd, const int64_t* lengths, float* P, float* Pdrop,
                            int64_t B, int64_t H, int64_t T, float scale, float dropout_p, const uint64_t* seed,
                            uint64_t rng_stream, void* stream);
int kdfm_relpos_softmax_bwd(const float* P, const float* dPdrop, float* dAC, float* dBD, int64_t B, int64_t H,
                            int64_t T, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                            void* stream);
/* sinusoidal table for relative positions T-1 ... -(T-1), (2T-1, d) */
int kdfm_relpos_table(float* pe, int64_t T, int64_t d, void* stream);
/* Fused relative-position MHA forward (bf16 MFMA): o[b,t,h*dk+c] = sum_j Pdrop[b,h,t,j] V[b,j,h*dk+c] with
 * scores ((q+u)K^T + rel_shift((q+v)Ppos^T)) * scale, key-padding mask from lengths, softmax,
 * inverted dropout (same counter-RNG mask as kdfm_relpos_softmax_fwd).  qu/qv/o: (B*T, d);
 * qkv: (B*T, 3d) (K at +d, V at +2d); pos: (2T-1, d) projected positions.  P / Pdrop (B,H,T,T) are
 * written when non-null (the per-op backward's operands; two passes over the keys); otherwise one
 * online-softmax pass, and lse (B,H,T) = per-row log-sum-exp of the scaled scores when non-null
 * (kdfm_relpos_attn_bwd's operand; 3e38 for rows without a valid key).  In the one-pass mode p_tilde
 * (B,H,T,T) bf16 = exp(s_ij - m_i,kb) before dropout and m_blk (B,H,T,ceil(T/64)) = the running row max
 * m_i,kb after key block kb are written when non-null (pairs with lse; entries at i or j >= length are not
 * written and not read).  dk = d/H <= 64.  K and V are centred before their bf16 rounding on kc / vc, the
 * mean of the utterance's first min(length, 16) (rounded down to a power of two) key / value rows: scores,
 * lse, p_tilde and m_blk are those of the centred keys (softmax is invariant; the backward kernels centre
 * identically) and O_i = sum_j Pdrop_ij (V_j - vc) + (sum_j Pdrop_ij) vc. */
int kdfm_relpos_attn_fwd(const float* qu, const float* qv, const float* qkv, const float* pos,
                         const int64_t* lengths, float* o, float* P, float* Pdrop, float* lse, uint16_t* p_tilde,
                         float* m_blk, int64_t B, int64_t H,
                         int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed,
                         uint64_t rng_stream, void* stream);
/* The same forward over PREPARED bf16 operands (csrc/attn_fwd3.hip; single pass, lse only -- the bwd2
 * backward's form -- or inference with lse NULL): the same bf16 operands, MFMAs and dropout mask as
 * kdfm_relpos_attn_fwd, its softmax in the exp2 domain (O within 1e-3, lse within 2e-6 of it).  Every operand
 * tile of a (64 queries, 64 keys) step is one contiguous range copied into LDS by LDS-DMA.
 *   kdfm_attn_kv_prep: kb / vb (B*H, Tp, LR) bf16 with Tp = T rounded up to 64, LR = DKP + 8, DKP = 48 (dk <= 48),
 *     64 (dk <= 64) or 128: rows j < T = bf16(K_j - kc) / bf16(V_j - vc) in columns < dk (the centring of
 *     kdfm_relpos_attn_fwd), zeros elsewhere; centre (B*H, 2, DKP) f32 = (kc, vc).  Sizes:
 *     kdfm_attn_kv_prep_elems / kdfm_attn_centre_elems (-1: unsupported).
 *   kdfm_attn_band_prep: every layer's projected positions pos + l * ld_layer ((2T-1, d) each) as pb
 *     (layers*H, NPB, LR) bf16, NPB = 64 + (2T-1) + 88, row 64 + r = position r, zeros around
 *     (kdfm_attn_band_prep_elems); kdfm_relpos_attn_fwd3 takes one layer's (H, NPB, LR) slice.
 * Replaces the per-layer attention call of NeMo RelPositionMultiHeadAttention (conformer_encoder.py:685-692,
 * Appendix A.7) like kdfm_relpos_attn_fwd; dk <= 128. */
int64_t kdfm_attn_kv_prep_elems(int64_t B, int64_t H, int64_t T, int64_t d);
int64_t kdfm_attn_centre_elems(int64_t B, int64_t H, int64_t d);
int64_t kdfm_attn_band_prep_elems(int64_t layers, int64_t H, int64_t T, int64_t d);
int kdfm_attn_kv_prep(const float* qkv, const int64_t* lengths, uint16_t* kb, uint16_t* vb, float* centre, int64_t B,
                      int64_t H, int64_t T, int64_t d, void* stream);
int kdfm_attn_band_prep(const float* pos, int64_t ld_layer, int64_t layers, uint16_t* pb, int64_t H, int64_t T,
                        int64_t d, void* stream);
/* bwd2 part 1 (kdfm_relpos_attn_bwd2_dq) over the forward's prepared operands: K / V / band tiles and the
 * centre from kdfm_attn_kv_prep / kdfm_attn_band_prep (the forward's own, kept for the backward) instead of
 * qkv / pos -- the same dqu / dqv / dS / Pd (DKP 64 / 128: dS and Pd bitwise, dqu / dqv up to the sign of zero
 * products; DKP 48: exp2-domain scores, dS / Pd within one bf16 rounding, dqu / dqv within 1e-3 relative). */
int kdfm_relpos_attn_bwd2_dq3(const float* dO, const float* O, const float* qu, const float* qv, const uint16_t* kb,
                              const uint16_t* vb, const float* centre, const uint16_t* pb, const float* lse,
                              const int64_t* lengths, uint16_t* ds, uint16_t* pd, float* dqu, float* dqv, int64_t B,
                              int64_t H, int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed,
                              uint64_t rng_stream, void* stream);
int kdfm_relpos_attn_fwd3(const float* qu, const float* qv, const uint16_t* kb, const uint16_t* vb, const float* centre,
                          const uint16_t* pb, const int64_t* lengths, float* o, float* lse, int64_t B, int64_t H,
                          int64_t T, int64_t d, float scale, float dropout_p, const uint64_t* seed, uint64_t rng_stream,
                          void* stream);
/* conv module: GLU over channels + pad mask; depthwise conv (k odd) with optional f64 BN stats */
int kdfm_glu_mask_fwd(const float* a, const int64_t* lengths, float* g, int64_t B, int64_t T, int64_t d,
                      void* stream);
int kdfm_glu_mask_bwd(const float* dg, const float* a, const int64_t* lengths, float* da, int64_t B, int64_t T,
                      int64_t d, void* stream);
/* The same with da rounded to bf16 (round to nearest even) for an operand only bf16-operand products read (the
 * large-tile GEMM's data and weight gradients of pointwise_conv1, FastConformer(-XL)). */
int kdfm_glu_mask_bwd_bf16(const float* dg, const float* a, const int64_t* lengths, uint16_t* da, int64_t B,
                           int64_t T, int64_t d, void* stream);
int kdfm_dwconv_fwd(const float* g, const float* w, const float* bias, float* y, double* stats, int64_t B, int64_t T,
                    int64_t d, int64_t K, void* stream);
/* dg = conv^T(dy); dw, db accumulate (+=) */
/* dw/db accumulated (+=) through per-block partials in ws (>= kdfm_dwconv_bwd_ws(B, T, d, K) floats);
 * dw == db == NULL: only dg, the partials are left in ws for kdfm_dwconv_bwd_fold (which may run on
 * another stream once this launch is complete -- the engine folds on the weight-gradient stream) */
int kdfm_dwconv_bwd(const float* dy, const float* g, const float* w, float* dg, float* dw, float* db, float* ws,
                    int64_t B, int64_t T, int64_t d, int64_t K, void* stream);
int kdfm_dwconv_bwd_fold(const float* ws, float* dw, float* db, int64_t B, int64_t T, int64_t d, int64_t K,
                         void* stream);
/* The BatchNorm(+SiLU) backward's elementwise half applied on load by the depthwise backward: dz is the
 * gradient wrt silu(BN(y)); red (2d doubles, zero before kdfm_bn_silu_bwd_reduce) holds the reduction's
 * sums (batch_stats: sum dyb | sum dyb xhat); the launch forms dy = d loss / d y tile by tile (never stored),
 * then dg and the weight partials as kdfm_dwconv_bwd (fold with kdfm_dwconv_bwd_fold); its first workgroup
 * adds the affine gradients dgamma += sum dyb xhat, dbeta += sum dyb and zeroes red_next (another 2d buffer
 * or NULL).  K = 15 or 31.  Replaces kdfm_bn_silu_bwd2's apply launch. */
int kdfm_dwconv_bwd_bn(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, const double* red, double* red_next, float* dgamma, float* dbeta,
                       int32_t batch_stats, const float* g, const float* w, float* dg, float* ws, int64_t B,
                       int64_t T, int64_t d, int64_t K, void* stream);
/* the BN-SiLU backward's reduction alone: red (2d doubles, zero on entry) += (sum dyb, sum dyb xhat) */
int kdfm_bn_silu_bwd_reduce(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                            const float* beta, double* red, int64_t rows, int64_t d, void* stream);
int64_t kdfm_dwconv_bwd_ws(int64_t B, int64_t T, int64_t d, int64_t K);
int kdfm_bn_finalize(const double* stats, const float* running_mean, const float* running_var, float* mean,
                     float* rstd, int64_t d, int64_t count, float eps, void* stream);
int kdfm_bn_running_update(float* running_mean, float* running_var, const double* stats, int64_t d, int64_t count,
                           float momentum, void* stream);
/* training step: kdfm_bn_finalize from the batch sums plus kdfm_bn_running_update in one launch; the
 * sums are reset to zero after they are read (a persistent stats buffer then serves the next layer's
 * kdfm_dwconv_fwd without a memset) */
int kdfm_bn_finalize_running(double* stats, float* running_mean, float* running_var, float* mean, float* rstd,
                             int64_t d, int64_t count, float eps, float momentum, void* stream);
int kdfm_bn_silu_fwd(const float* y, const float* mean, const float* rstd, const float* gamma, const float* beta,
                     float* z, int64_t rows, int64_t d, void* stream);
/* z rounded to bf16 (the large-tile pointwise_conv2 and its weight gradient read bf16 operands). */
int kdfm_bn_silu_fwd_bf16(const float* y, const float* mean, const float* rstd, const float* gamma, const float* beta,
                          uint16_t* z, int64_t rows, int64_t d, void* stream);
int kdfm_bn_silu_bwd(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, double* red_ws, float* dy, float* dgamma, float* dbeta, int64_t rows,
                     int64_t d, int32_t batch_stats, void* stream);
/* the same without the memset: red_ws (2d doubles) must be zero on entry; red_next (another 2d buffer or
 * NULL) is zeroed by the launch for the next call -- a ring of buffers serves a stack of layers */
int kdfm_bn_silu_bwd2(const float* dz, const float* y, const float* mean, const float* rstd, const float* gamma,
                      const float* beta, double* red_ws, double* red_next, float* dy, float* dgamma, float* dbeta,
                      int64_t rows, int64_t d, int32_t batch_stats, void* stream);

/* ---------------- decoder / losses (conv_asr.py:456-468; losses/ctc.py:68-82; asr_train_diffm.py:740-811) */
int kdfm_log_softmax(const float* x, float* y, int64_t rows, int64_t C, int64_t ldx, int64_t ldy, void* stream);
/* idx[r] = argmax_c x[r, c] (first maximum) — greedy CTC predictions */
int kdfm_argmax_rows(const float* x, int64_t* idx, int64_t rows, int64_t C, void* stream);
/* dx = dy - exp(y) * rowsum(dy), y the log_softmax output (contiguous rows of C) */
int kdfm_log_softmax_bwd(const float* dy, const float* y, float* dx, int64_t rows, int64_t C, void* stream);
/* per-utterance CTC NLL and d(grad_scale * nll)/dlogits = grad_scale*(exp(lp) - posterior) */
int kdfm_ctc_loss(const float* log_probs, const int64_t* targets, const int64_t* input_lengths,
                  const int64_t* target_lengths, float* alpha_ws, float* beta_ws, float* nll, float* grad, int64_t B,
                  int64_t T, int64_t C, int64_t Umax, int64_t blank, float grad_scale, int32_t zero_infinity,
                  void* stream);
/* KL(softmax(t/T) || log_softmax(s/T)); grad += grad_coef*(softmax(s/T) - p_t); *loss_acc += loss_scale*KL */
int kdfm_kl_div_logits(const float* student_logp, const float* teacher_logits, float* grad, float* loss_acc,
                       int64_t rows, int64_t C, float temperature, float grad_coef, float loss_scale, void* stream);
/* out5 = [total, ctc(mean_batch), kl, recon, fm] */
int kdfm_loss_combine(const float* nll, int64_t B, const float* kl, const float* recon, const float* fm,
                      float kd_alpha, float* out5, void* stream);

/* ---------------- ver5 KD heads (asr_train_diffm.py:400-497, 1270-1427) -------------------- */
int kdfm_adapter_fwd(const float* zs, const float* h, const float* w2, const float* b2, const float* eps_in, float* zn,
                     float* gamma, int64_t rows, int64_t L, const uint64_t* seed, uint64_t rng_stream, void* stream);
/* NoiseAdapter backward: dzs, dh per row; dw2 += sum dgl h, db2 += sum dgl through per-workgroup partials in
 * ws (kdfm_adapter_bwd_ws floats) folded in a fixed order (deterministic).  L a multiple of 16, <= 128. */
int64_t kdfm_adapter_bwd_ws(int64_t rows, int64_t L);
int kdfm_adapter_bwd(const float* dzn, const float* zs, const float* h, const float* gamma, const float* w2,
                     const float* eps_in, float* dzs, float* dh, float* dw2, float* db2, float* ws, int64_t ws_len,
                     int64_t rows, int64_t L, const uint64_t* seed, uint64_t rng_stream, void* stream);
int kdfm_fm_step_bias(const float* w_te, const float* b_te, const float* W1, const float* b1, float* cvec, float* evec,
                      int64_t L, int64_t E, int64_t steps, void* stream);
int kdfm_fm_time_bwd(const float* dc, const float* evec, const float* W1, float* dW1, float* db1, float* dw_te,
                     float* db_te, int64_t L, int64_t E, int64_t steps, void* stream);

/* ---------------- glue ------------------------------------------------------------------ */
int kdfm_fill(float* x, float value, int64_t n, void* stream);
int kdfm_axpby(const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int64_t ldo, int64_t rows,
               int64_t cols, float alpha, float beta, void* stream);
int kdfm_dropout(const float* x, float* out, int64_t n, float p, float scale, const uint64_t* seed,
                 uint64_t rng_stream, void* stream);
/* The same with out rounded to bf16 (the residual-branch dropout gradients the large-tile data and weight gradients
 * read: one bf16 operand instead of an f32 tensor cast per consumer). */
int kdfm_dropout_bf16(const float* x, uint16_t* out, int64_t n, float p, float scale, const uint64_t* seed,
                      uint64_t rng_stream, void* stream);
/* out[r,c] = alpha * x[r,c] * s[r / rows_per_s]  (s: device scalars, e.g. upstream loss grads) */
int kdfm_rowscale(const float* x, float* out, int64_t rows, int64_t cols, const float* s, int64_t rows_per_s,
                  float alpha, void* stream);
/* out = (y > 0) ? dy : 0 */
int kdfm_relu_mask(const float* dy, const float* y, float* out, int64_t n, void* stream);
/* nn.MSELoss pieces: *loss_acc += scale * sum (a-b)^2 ; grad = gscale * (a-b) when grad != NULL */
int kdfm_mse(const float* a, const float* b, float* grad, float* loss_acc, int64_t n, float scale, float gscale,
             void* stream);
/* nn.L1Loss pieces (kd_crit, kd_loss_type "l1": asr_train_diffm.py:557, used by versions 1/3/4/8 at
 * :675-727): *loss_acc += scale * sum |a-b| ; grad = gscale * sign(a-b) when grad != NULL */
int kdfm_l1(const float* a, const float* b, float* grad, float* loss_acc, int64_t n, float scale, float gscale,
            void* stream);
/* NeMo Conv1d weight (O,I,K) -> fwd (O,K,I) and transposed+flipped bwd (I,K,O) GEMM layouts */
/* Strided 1-D unfold / fold over channels-last rows of B utterances (csrc/unfold.hip), for the U-Net FM
 * meta-encoder (asr_train.py:880-917: Conv1d(k 4, s 2, p 1) downs = unfold + GEMM; ConvTranspose1d(k 4, s 2,
 * p 1) ups = GEMM + fold; their data gradients the other way round).
 *   kdfm_unfold1d: cols[(b, i)][k C + c] = x[(b, S i - P + k)][c] for i < Lrows (0 outside [0, Lvalid)); utterance
 *     b's rows start at row b Lin (Lvalid <= Lin), x rows of stride ldx.
 *   kdfm_fold1d: out[(b, t)][c] = R[(b, t)][c] (when non-null, may alias out) + [t < Lvalid] (bias[c] (when
 *     non-null) + sum over taps k with t + P - k = S i, 0 <= i < Lrows, of cols[(b, i)][k C + c]), for t < Lout
 *     (Lvalid: a transposed conv's own output length -- taps past it are cropped, rows past it the zero pad).
 * C, ldx, ldo, ldr multiples of 4; K <= 16. */
int kdfm_unfold1d(const float* x, int64_t ldx, float* cols, int64_t B, int64_t Lin, int64_t Lvalid, int64_t Lrows,
                  int64_t C, int32_t K, int32_t S, int32_t P, void* stream);
int kdfm_fold1d(const float* cols, float* out, int64_t ldo, const float* bias, const float* R, int64_t ldr, int64_t B,
                int64_t Lrows, int64_t Lout, int64_t Lvalid, int64_t C, int32_t K, int32_t S, int32_t P, void* stream);
int kdfm_convw_prep(const float* W, float* fwd, float* bwd, int64_t O, int64_t I, int64_t K, void* stream);
/* dW(O,I,K) += alpha * G(O,K,I) */
int kdfm_convw_grad(const float* G, float* dW, int64_t O, int64_t I, int64_t K, float alpha, void* stream);
/* mel_len = wav_len // hop (FilterbankFeatures.get_seq_len); len1/len2 after each striding conv
 * (ConvSubsampling calc_length: floor((l + 2*1 - 3)/2 + 1)) */
int kdfm_subsample_lengths(const int64_t* wav_len, int64_t* mel_len, int64_t* len1, int64_t* len2, int64_t B,
                           int64_t hop, void* stream);
/* step counter += 1 and per-step RNG seed advance, on device */
int kdfm_step_advance(int64_t* step, uint64_t* seed, void* stream);

/* ---------------- optimizer (modelPT.py:650-897, lr_scheduler.py:473-530) ------------------
 * step[0] = k, the 1-based optimizer step (Noam schedule); AdamW's bias correction counts
 * k - adam_base[0] (adam_base may be NULL = 0): the moments restarted adam_base steps into the run
 * (a resume whose optimizer state could not be restored), like a fresh torch AdamW state.
 * gstats (optional, kdfm_grad_stats' output): when gstats[1] != 0 the gradient holds a non-finite
 * value and the update is skipped (parameters and moments unchanged; the schedule step still counts,
 * lr_out still written) and adam_base[0] += 1, so AdamW's bias correction counts only the steps that
 * updated the moments (torch's AdamW `step` semantics).  The reference has no such check (Lightning's
 * default); it is opt-in (Ver5Config.grad_check). */
int kdfm_adamw_noam(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                    const int64_t* step, int64_t* adam_base, float base_lr, float d_model,
                    float warmup_steps, float min_lr, float beta1, float beta2, float eps, float weight_decay,
                    float grad_scale, float* lr_out, const float* gstats, void* stream);
/* The same update also writing the new parameters as bf16 (round to nearest even) into params_bf16, a mirror of the
 * flat buffer the large-tile GEMM reads its weight operands from (FastConformer(-XL): no per-weight cast per step). */
int kdfm_adamw_noam_bf16(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, uint16_t* params_bf16,
                         int64_t n, const int64_t* step, int64_t* adam_base, float base_lr, float d_model,
                         float warmup_steps, float min_lr, float beta1, float beta2, float eps, float weight_decay,
                         float grad_scale, float* lr_out, const float* gstats, void* stream);
/* out2 = [sum_i (scale g_i)^2 over the finite entries, number of non-finite entries] of the flat gradient
 * buffer (the all-reduced sum with scale = 1/world: the global gradient norm^2 and the
 * skip flag of kdfm_adamw_noam); fixed-order two-stage reduction (deterministic).  ws: kdfm_grad_stats_ws
 * floats. */
int64_t kdfm_grad_stats_ws(void);
int kdfm_grad_stats(const float* grads, int64_t n, float scale, float* ws, int64_t ws_len, float* out2,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KDFM_H_ */
