# knockout what-if probe (kdfm/plan.py KDFM_PLAN_KNOCKOUT): the step time with one kernel family's launches
# dropped from the replayed plan -- an upper bound on what speeding that family up can buy
set -o pipefail
OUT=gpurun_out/r5zg
mkdir -p $OUT
run() {
  KDFM_PLAN_KNOCKOUT="$1" timeout -k 10 200 python3 -u bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1
  rc=$?
  # a Python error (rc 1) is reported and the probe goes on; a crash, abort or time limit ends the call
  [ $rc -le 1 ] || { echo "run died ($rc): $1"; tail -5 $OUT/run.log; exit 3; }
  [ $rc -eq 0 ] || { echo "run failed: $1"; tail -2 $OUT/run.log; }
  grep KNOCKOUT $OUT/run.log || tail -1 $OUT/run.log | cut -c1-200
}
run ""
run kdfm_wgrad_bf16,kdfm_wgrad_bf16_pair,kdfm_wgrad_fold_flush,kdfm_wgrad_bf16_seg,kdfm_wgrad_bf16_conv
run kdfm_relpos_attn_fwd3,kdfm_attn_kv_prep
run kdfm_relpos_attn_bwd2_dq3,kdfm_relpos_attn_bwd2_dkv,kdfm_relpos_attn_bwd2_dpos
run kdfm_ffn_fwd
run kdfm_ffn_bwd
run kdfm_ln_qkv_fwd,kdfm_ln_glu_fwd,kdfm_rowgemm
run kdfm_logmel_fft,kdfm_subsample_fused,kdfm_preemph_pad,kdfm_logmel_normalize,kdfm_specaugment
run kdfm_subsample_conv2_dgrad_w0_h,kdfm_ss_out_dgrad,kdfm_im2col_3x3s2_tm_bf16
run kdfm_fm_chain_fwd,kdfm_fm_chain_bwd,kdfm_denoise_chain_fwd,kdfm_denoise_chain_bwd
run kdfm_ctc_loss,kdfm_kl_div_logits
run kdfm_dwconv_fwd,kdfm_dwconv_bwd_bn,kdfm_bn_silu_bwd_reduce
run kdfm_gemm
run ""
