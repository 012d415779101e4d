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
  KDFM_EPI_ATOMIC = 1 << 9     /* atomicAdd into C (split-K reductions; no other epi)   */
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
} kdfm_gemm_desc;

int kdfm_gemm(const kdfm_gemm_desc* d, void* stream);

/* column sums: out[n] (+)= sum_m X[m*ld + n], m < M; accumulate != 0 adds into out.
 * (bias gradients of every Linear / Conv1d on the path) */
int kdfm_colsum(const float* X, float* out, int64_t M, int64_t N, int64_t ld, int32_t accumulate,
                void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KDFM_H_ */
