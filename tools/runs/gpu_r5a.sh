# round 5 first GPU pass: head-dim-128 attention kernels vs float64, the prepared-operand forward (fwd3) bitwise
# vs the register-staged one, the meta-encoder workspace test, the XL step-parity cases, then the bench line
set -o pipefail
OUT=gpurun_out/r5a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attn_fwd3_gpu.py \
  tests/test_attn_bwd_gpu.py tests/test_attn_fused_gpu.py "tests/test_encfm_meta_gpu.py::test_meta_workspace_follows_batch_shape" "tests/test_encfm_meta_gpu.py::test_conformer_meta_dropout_gradient_matches_finite_differences" \
  tests/test_step_parity_gpu.py -k "fwd3 or dq3 or prepared or head_dim or bwd or fused or workspace or dropout_gradient or xl or 2L-1.2s-dw4 or conformer-small" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
KDFM_ATTN_DQ3=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_nodq3.log 2>&1 || { tail -5 $OUT/bench_nodq3.log; exit 3; }
tail -1 $OUT/bench_nodq3.log | cut -c1-300
KDFM_ATTN_FWD3=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_nofwd3.log 2>&1 || { tail -5 $OUT/bench_nofwd3.log; exit 3; }
tail -1 $OUT/bench_nofwd3.log | cut -c1-300
exit $rc
