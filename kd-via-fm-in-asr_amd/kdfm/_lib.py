"""ctypes binding of libkdfm.so (include/kdfm.h).

The library is loaded AFTER torch so that its DT_NEEDED libamdhip64.so.7 resolves to the HIP
runtime torch already mapped (one runtime per process: torch streams are valid in our calls).
There is no fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must be imported first, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkdfm.so")
# experiment builds (tools/): an alternative in-tree library, e.g. a kernel-variant sweep
LIB_PATH = os.environ.get("KDFM_LIB") or LIB_PATH

KDFM_MATH_F32 = 0
KDFM_MATH_BF16 = 1

LD_KC, LD_XC, LD_CONV = 0, 1, 2
BIG_NT, BIG_NN, BIG_TN = 0, 1, 2   # kdfm_gemm_big operand layouts (include/kdfm.h KDFM_BIG_*)

EPI_BIAS = 1 << 0
EPI_STORE_PRE = 1 << 1
EPI_RELU = 1 << 2
EPI_SILU = 1 << 3
EPI_DROPOUT = 1 << 4
EPI_DRELU = 1 << 5
EPI_DSILU = 1 << 6
EPI_RESID = 1 << 7
EPI_BETA = 1 << 8
EPI_ATOMIC = 1 << 9
EPI_ROWMASK = 1 << 10
EPI_MSE = 1 << 11

_i64 = C.c_int64
_i32 = C.c_int32
_f32 = C.c_float
_vp = C.c_void_p


class GemmDesc(C.Structure):
    _fields_ = [
        ("A", _vp), ("B", _vp), ("C", _vp), ("bias", _vp), ("R", _vp), ("aux", _vp), ("Cpre", _vp),
        ("M", _i64), ("N", _i64), ("K", _i64),
        ("sAm", _i64), ("sAk", _i64), ("sBk", _i64), ("sBn", _i64), ("sCm", _i64), ("sCn", _i64),
        ("batch1", _i64), ("batch2", _i64),
        ("bA1", _i64), ("bA2", _i64), ("bB1", _i64), ("bB2", _i64), ("bC1", _i64), ("bC2", _i64),
        ("alpha", _f32), ("beta", _f32), ("rscale", _f32), ("dropout_p", _f32),
        ("seed", _vp), ("rng_stream", C.c_uint64),
        ("amode", _i32), ("bmode", _i32), ("epi", _i32), ("math", _i32),
        ("splitk", _i32),
        ("conv_taps", _i32), ("conv_pad", _i32),
        ("conv_c", _i64), ("conv_t", _i64),
        ("mask_len", _vp), ("mask_T", _i64), ("mask_div", _i64),
        ("loss_acc", _vp), ("loss_scale", _f32),
        ("ones_out", _vp), ("ones_col", _i64),
        ("ws", _vp), ("ws_len", _i64),
        ("Bh", _vp), ("sBh", _i64),
    ]


# Every symbol include/kdfm.h declares, with its ctypes signature.  tests/test_abi.py checks this
# table against the header so the two cannot drift.
P = _vp
SIGNATURES: dict[str, tuple] = {
    "kdfm_version": (C.c_char_p, []),
    "kdfm_last_error": (C.c_char_p, []),
    "kdfm_device_arch": (_i32, [C.c_char_p, _i64]),
    "kdfm_set_deterministic": (None, [_i32]),
    "kdfm_get_deterministic": (_i32, []),
    "kdfm_gemm": (_i32, [C.POINTER(GemmDesc), P]),
    "kdfm_gemm_ws": (_i64, [C.POINTER(GemmDesc)]),
    "kdfm_gemm_last_route": (_i32, []),
    "kdfm_range_push": (_i32, [C.c_char_p]),
    "kdfm_wgrad_bf16_ws": (_i64, [_i64, _i64, _i64, _i32]),
    "kdfm_relpos_attn_bwd_ws": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_relpos_attn_bwd": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _f32, _f32, P,
                                    C.c_uint64, P]),
    "kdfm_attn_kv_prep_elems": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_attn_centre_elems": (_i64, [_i64, _i64, _i64]),
    "kdfm_attn_band_prep_elems": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_attn_kv_prep": (_i32, [P, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_attn_band_prep": (_i32, [P, _i64, _i64, P, _i64, _i64, _i64, P]),
    "kdfm_relpos_attn_bwd2_dq3": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _f32, _f32, P,
                                         C.c_uint64, P]),
    "kdfm_relpos_attn_fwd3": (_i32, [P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_unfold1d": (_i32, [P, _i64, P, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, P]),
    "kdfm_fold1d": (_i32, [P, P, _i64, P, P, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, P]),
    "kdfm_relpos_attn_bwd2_ldt": (_i64, [_i64]),
    "kdfm_relpos_attn_bwd2_dpos_ws": (_i64, [_i64, _i64, _i64]),
    "kdfm_relpos_attn_bwd2_dq": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _f32, _f32, P,
                                        C.c_uint64, P]),
    "kdfm_relpos_attn_bwd2_dkv": (_i32, [P, P, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_relpos_attn_bwd2_dpos": (_i32, [P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, P]),
    "kdfm_relpos_attn_bwd_parts": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _f32,
                                          _f32, P, C.c_uint64, _i32, P]),
    "kdfm_wgrad_bf16": (_i32, [P, P, P, _i64, P, _i64, _i64, _i64, _f32, P, _i64, P]),
    "kdfm_wgrad_bf16_pair": (_i32, [P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _f32, P, _i64, P]),
    "kdfm_fm_chain_fwd": (_i32, [P, P, P, _i64, P, P, P, P, P, P, P, P, P, P, P, _f32, _i64, _i32, _i32, P]),
    "kdfm_rowgemm_img_elems": (_i64, [_i64]),
    "kdfm_wimg_job_threads": (_i64, [P]),
    "kdfm_wimg_prep_batch": (_i32, [P, _i32, _i64, P]),
    "kdfm_rowgemm_wprep": (_i32, [P, P, _i64, _i32, P]),
    "kdfm_rowgemm": (_i32, [P, P, P, _i64, _i64, _i32, _f32, _f32, C.c_uint64, P, P, P, P, P, _i32, P, P, _f32, _f32,
                            C.c_uint64, P, P]),
    "kdfm_lnproj_img_elems": (_i64, [_i32, _i64, _i32]),
    "kdfm_lnproj_wprep": (_i32, [_i32, P, P, _i64, _i32, P]),
    "kdfm_ln_qkv_fwd": (_i32, [P, P, P, _f32, P, P, P, P, P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_ln_glu_fwd": (_i32, [P, P, P, _f32, P, P, P, _i64, P, P, P, P, _i64, _i64, P]),
    "kdfm_ln_qkv_bwd": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_ln_glu_bwd": (_i32, [P, P, P, P, P, P, P, P, P, _i64, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_ffn_supported": (_i32, [_i64, _i64]),
    "kdfm_ffn_img_elems": (_i64, [_i64, _i64]),
    "kdfm_ffn_wprep": (_i32, [P, P, P, _i64, _i64, _i32, P]),
    "kdfm_ffn_fwd": (_i32, [P, P, P, _f32, P, P, P, P, P, P, _i64, _i64, _i64, _f32, _f32, _f32, P, C.c_uint64,
                            C.c_uint64, P, P, _f32, P, P, P, P]),
    "kdfm_ffn_bwd": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _f32, _f32, _f32, P,
                            C.c_uint64, C.c_uint64, P]),
    "kdfm_fm_chain_bwd": (_i32, [P, P, P, P, _i64, P, P, P, P, P, _i64, _i32, _i32, P]),
    "kdfm_wgrad_bf16_seg_ws": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_wgrad_bf16_seg": (_i32, [P, P, P, _i64, P, _i64, _i64, _i64, _i64, _f32, P, _i64, P]),
    "kdfm_wgrad_bf16_conv_ws": (_i64, [_i64, _i64, _i64, _i32, _i32, _i64, _i32]),
    "kdfm_wgrad_bf16_s2conv_ws": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_wgrad_bf16_s2conv": (_i32, [P, P, _i64, P, P, P, _i64, _i64, _i64, _i64, _f32, P, _i64, P]),
    "kdfm_wgrad_bf16_conv": (_i32, [P, P, P, _i64, P, _i64, _i64, _i64, _i32, _i32, _i64, _f32, P, _i64, P]),
    "kdfm_wgrad_set_fold_arena": (_i32, [P, P, _i64]),
    "kdfm_wgrad_fold_flush": (_i32, [P]),
    "kdfm_wgrad_fold_pending": (_i64, [P]),
    "kdfm_wgrad_fold_stats": (_i32, [P, P]),
    "kdfm_wgrad_fold_discard_all": (_i32, []),
    "kdfm_denoise_wimg_elems": (_i64, []),
    "kdfm_subsample_dgrad_wprep_elems": (_i64, [_i64]),
    "kdfm_subsample_dgrad_wprep": (_i32, [P, P, _i64, P]),
    "kdfm_subsample_conv2_dgrad": (_i32, [P, P, P, P, _i64, _i64, _i64, _i64, _i64, P]),
    "kdfm_subsample_conv2_dgrad_w0_ws": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_subsample_conv2_dgrad_w0": (_i32, [P, P, P, P, _i64, _i64, _i64, _i64, _i64, P, P, _i64, _i64, _i64, P, P, P,
                                              _i64, P]),
    "kdfm_subsample_conv2_dgrad_w0_h": (_i32, [P, P, P, P, _i64, _i64, _i64, _i64, _i64, P, P, _i64, _i64, _i64, P, P, P,
                                                _i64, P]),
    "kdfm_ss_out_wprep_elems": (_i64, [_i64, _i64]),
    "kdfm_ss_out_wprep": (_i32, [P, P, _i64, _i64, P]),
    "kdfm_ss_out_dgrad": (_i32, [P, P, P, P, _i64, _i64, _i64, P]),
    "kdfm_denoise_chain_fwd": (_i32, [P, P, P, P, P, P, P, P, P, _i64, _i64, _i32, _i32, P]),
    "kdfm_denoise_chain_bwd": (_i32, [P, P, P, P, P, P, P, P, _i64, _i64, _i32, _i32, P]),
    "kdfm_range_pop": (_i32, []),
    "kdfm_event_record": (_i32, [P, P]),
    "kdfm_stream_wait_event": (_i32, [P, P]),
    "kdfm_event_create": (_i32, [P, C.c_uint32]),
    "kdfm_event_destroy": (_i32, [P]),
    "kdfm_stream_create_cu_mask": (_i32, [_i32, C.POINTER(C.c_void_p)]),
    "kdfm_memset_async": (_i32, [P, _i32, _i64, P]),
    "kdfm_cast_bf16": (_i32, [P, P, _i64, P]),
    "kdfm_cast_bf16_2d": (_i32, [P, _i64, P, _i64, _i64, _i64, P]),
    "kdfm_gemm_big_supported": (_i32, [_i64, _i64, _i64, _i32]),
    "kdfm_gemm_big_ws": (_i64, [_i64, _i64, _i64, _i32]),
    "kdfm_fp8_quant_mx": (_i32, [P, _i32, _i64, _i64, _i64, P, _i64, P, _i32, P]),
    "kdfm_gemm_big_fp8": (_i32, [C.POINTER(GemmDesc), P, _i64, P, _i64, P, P, P, P]),
    "kdfm_gemm_big": (_i32, [C.POINTER(GemmDesc), P, _i64, P, _i64, _i32, P, P]),
    "kdfm_cast_bf16_t": (_i32, [P, P, P, _i64, _i64, P]),
    "kdfm_colsum": (_i32, [P, P, _i64, _i64, _i64, _f32, _i32, P]),
    "kdfm_preemph_pad": (_i32, [P, P, P, _i64, _i64, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_power_spectrum": (_i32, [P, P, _i64, _i64, P]),
    "kdfm_logmel_fft": (_i32, [P, _i64, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _i64, P]),
    "kdfm_logmel_normalize": (_i32, [P, P, P, _i64, _i64, _i64, _f32, P]),
    "kdfm_specaugment": (_i32, [P, P, P, _i64, _i64, _i64, _i32, _i32, _i32, _f32, P, C.c_uint64, P, P]),
    "kdfm_im2col_3x3s2": (_i32, [P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_im2col_3x3s2_tm_bf16": (_i32, [P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_im2col_3x3s2_tm_from_bf16": (_i32, [P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_conv_lengths": (_i32, [P, P, _i64, _i32, _i32, _i32, P]),
    "kdfm_dwsub_conv": (_i32, [P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, P]),
    "kdfm_dwsub_conv_dgrad": (_i32, [P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, P]),
    "kdfm_dwsub_conv_wgrad_ws": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_dwsub_conv_wgrad": (_i32, [P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32,
                                      _i32, P]),
    "kdfm_col2im_3x3s2": (_i32, [P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_col2im_3x3s2_tapmajor": (_i32, [P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_subsample_wprep_elems": (_i64, [_i64]),
    "kdfm_subsample_wprep": (_i32, [P, P, _i64, P]),
    "kdfm_subsample_conv1": (_i32, [P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_subsample_conv2": (_i32, [P, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_subsample_fused_supported": (_i32, [_i64, _i64]),
    "kdfm_subsample_fused_wprep_elems": (_i64, [_i64]),
    "kdfm_subsample_fused_wprep": (_i32, [P, P, P, _i64, P]),
    "kdfm_subsample_fused": (_i32, [P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, P]),
    "kdfm_ctc_greedy": (_i32, [P, _i64, P, P, P, P, _i64, _i64, _i64, _i64, _i32, P]),
    "kdfm_edit_distance": (_i64, [P, _i64, P, _i64]),
    "kdfm_layernorm_fwd": (_i32, [P, P, P, P, P, P, _i64, _i64, _f32, P]),
    "kdfm_layernorm_fwd_bf16": (_i32, [P, P, P, P, P, P, _i64, _i64, _f32, P]),
    "kdfm_layernorm_bwd": (_i32, [P, P, P, P, P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_layernorm_bwd_ws": (_i64, [_i64, _i64]),
    "kdfm_layernorm_bwd_part": (_i32, [P, P, P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_layernorm_bwd_part2": (_i32, [P, P, P, P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_ln_fold": (_i32, [C.POINTER(P), C.POINTER(P), C.POINTER(P), _i32, _i64, _i64, P]),
    "kdfm_qkv_prep": (_i32, [P, P, P, P, P, _i64, _i64, P]),
    "kdfm_relpos_softmax_fwd": (_i32, [P, P, P, P, P, _i64, _i64, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_relpos_softmax_bwd": (_i32, [P, P, P, P, _i64, _i64, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_relpos_attn_fwd": (_i32, [P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_relpos_table": (_i32, [P, _i64, _i64, P]),
    "kdfm_glu_mask_fwd": (_i32, [P, P, P, _i64, _i64, _i64, P]),
    "kdfm_glu_mask_bwd": (_i32, [P, P, P, P, _i64, _i64, _i64, P]),
    "kdfm_glu_mask_bwd_bf16": (_i32, [P, P, P, P, _i64, _i64, _i64, P]),
    "kdfm_dwconv_fwd": (_i32, [P, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_dwconv_bwd": (_i32, [P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_dwconv_bwd_fold": (_i32, [P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_dwconv_bwd_bn": (_i32, [P, P, P, P, P, P, P, P, P, P, _i32, P, P, P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_bn_silu_bwd_reduce": (_i32, [P, P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_dwconv_bwd_ws": (_i64, [_i64, _i64, _i64, _i64]),
    "kdfm_bn_finalize": (_i32, [P, P, P, P, P, _i64, _i64, _f32, P]),
    "kdfm_bn_running_update": (_i32, [P, P, P, _i64, _i64, _f32, P]),
    "kdfm_bn_finalize_running": (_i32, [P, P, P, P, P, _i64, _i64, _f32, _f32, P]),
    "kdfm_bn_silu_fwd": (_i32, [P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_bn_silu_fwd_bf16": (_i32, [P, P, P, P, P, P, _i64, _i64, P]),
    "kdfm_bn_silu_bwd": (_i32, [P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i32, P]),
    "kdfm_bn_silu_bwd2": (_i32, [P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i32, P]),
    "kdfm_log_softmax": (_i32, [P, P, _i64, _i64, _i64, _i64, P]),
    "kdfm_argmax_rows": (_i32, [P, P, _i64, _i64, P]),
    "kdfm_log_softmax_bwd": (_i32, [P, P, P, _i64, _i64, P]),
    "kdfm_ctc_loss": (_i32, [P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i64, _i64, _f32, _i32, P]),
    "kdfm_kl_div_logits": (_i32, [P, P, P, P, _i64, _i64, _f32, _f32, _f32, P]),
    "kdfm_loss_combine": (_i32, [P, _i64, P, P, P, _f32, P, P]),
    "kdfm_adapter_fwd": (_i32, [P, P, P, P, P, P, P, _i64, _i64, P, C.c_uint64, P]),
    "kdfm_adapter_bwd_ws": (_i64, [_i64, _i64]),
    "kdfm_adapter_bwd": (_i32, [P, P, P, P, P, P, P, P, P, P, P, _i64, _i64, _i64, P, C.c_uint64, P]),
    "kdfm_fm_step_bias": (_i32, [P, P, P, P, P, P, _i64, _i64, _i64, P]),
    "kdfm_fm_time_bwd": (_i32, [P, P, P, P, P, P, P, _i64, _i64, _i64, P]),
    "kdfm_fill": (_i32, [P, _f32, _i64, P]),
    "kdfm_axpby": (_i32, [P, _i64, P, _i64, P, _i64, _i64, _i64, _f32, _f32, P]),
    "kdfm_rowscale": (_i32, [P, P, _i64, _i64, P, _i64, _f32, P]),
    "kdfm_relu_mask": (_i32, [P, P, P, _i64, P]),
    "kdfm_mse": (_i32, [P, P, P, P, _i64, _f32, _f32, P]),
    "kdfm_l1": (_i32, [P, P, P, P, _i64, _f32, _f32, P]),
    "kdfm_dropout": (_i32, [P, P, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_dropout_bf16": (_i32, [P, P, _i64, _f32, _f32, P, C.c_uint64, P]),
    "kdfm_convw_prep": (_i32, [P, P, P, _i64, _i64, _i64, P]),
    "kdfm_convw_grad": (_i32, [P, P, _i64, _i64, _i64, _f32, P]),
    "kdfm_subsample_lengths": (_i32, [P, P, P, P, _i64, _i64, P]),
    "kdfm_step_advance": (_i32, [P, P, P]),
    "kdfm_adamw_noam": (_i32, [P, P, P, P, _i64, P, P, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _f32, P, P, P]),
    "kdfm_adamw_noam_bf16": (_i32, [P, P, P, P, P, _i64, P, P, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _f32, P, P,
                                    P]),
    "kdfm_wgrad_bf16_dev": (_i32, [P, P, P, _i64, P, _i64, P, _i64, _i64, _f32, P, _i64, P]),
    "kdfm_encfm_time_prep": (_i32, [P, _i64, P, P, P, _i32, _i32, _i32, P, P]),
    "kdfm_encfm_router_fwd": (_i32, [P, P, P, P, P, P, P, P, P, P, P, P, P, C.c_uint64, _i32, P, P, P, P, P, P, P,
                                     _i64, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _i32, P]),
    "kdfm_encfm_strategy": (_i32, [P, P, P, P, P, P, P, P, _i64, _i64, _i64, _i32, _i32, _i32, _f32, _f32, _f32,
                                   _i32, P]),
    "kdfm_encfm_chain_fwd": (_i32, [P, P, P, P, P, P, _i64, P, P, P, P, P, P, P, _i32, P, P, P, P, P, _i64, P,
                                    _i64, _i64, _i64, _i32, _i32, P]),
    "kdfm_encfm_chain_bwd": (_i32, [P, P, P, _i64, P, P, P, _i64, P, P, P, P, _i32, P, P, P, P, _i64, _i64, _i64,
                                    _i32, _i32, P]),
    "kdfm_encfm_router_bwd": (_i32, [P, P, P, P, P, P, _f32, P, P, P, P, _i64, _i64, _i32, _i32, P]),
    "kdfm_encfm_time_bwd": (_i32, [P, _i64, P, P, P, P, P, P, P, P, _i64, _i64, _i32, P]),
    "kdfm_grad_stats_ws": (_i64, []),
    "kdfm_grad_stats": (_i32, [P, _i64, _f32, P, _i64, P, P]),
}

_LIB = None


class KdfmError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise KdfmError(f"libkdfm.so not built ({LIB_PATH}); run __graft_entry__.build()")
        h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = h
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().kdfm_last_error().decode(errors="replace")
        raise KdfmError(f"{what} failed (status {rc}): {msg}")


_FN: dict = {}


def call(name: str, *args) -> None:
    fn = _FN.get(name)
    if fn is None:
        fn = _FN[name] = getattr(lib(), name)
    rc = fn(*args)
    if rc:
        check(rc, name)
