# bwd2 dQ epilogue rework (lane-permute skew, exp2, shared pair hashes, transposed dS / Pd tiles): attention tests,
# step parity, bwd2 micro (before: git stash build not kept -- compare with r5d's 64 us in-step), bench
set -o pipefail
OUT=gpurun_out/r5y
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attn_fwd3_gpu.py tests/test_attn_bwd_gpu.py tests/test_attn_fused_gpu.py tests/test_step_parity_gpu.py tests/test_encfm_meta_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 200 python3 -u tools/attn_bwd2_micro.py > $OUT/bwd2.log 2>&1 || { echo "micro failed"; tail -5 $OUT/bwd2.log; exit 3; }
cat $OUT/bwd2.log
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b.log; exit 3; }
  tail -1 $OUT/b.log | cut -c1-120
done
exit $rc
