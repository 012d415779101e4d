# round 5 second GPU pass: the prepared-operand attention fix (bit_cast of a vector element), head-dim-128
# kernels, the unet meta-encoder and the meta-encoder tests, the XL step parity, then bench A/Bs
set -o pipefail
OUT=gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg/fwd3_dbg.py > $OUT/fwd3_dbg.log 2>&1 || { tail -5 $OUT/fwd3_dbg.log; exit 2; }
cat $OUT/fwd3_dbg.log | grep rows
timeout -k 10 700 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attn_fwd3_gpu.py \
  tests/test_attn_bwd_gpu.py tests/test_attn_fused_gpu.py tests/test_encfm_meta_gpu.py \
  tests/test_step_parity_gpu.py -k "fwd3 or dq3 or prepared or head_dim or bwd or fused or meta or unet or xl or 2L-1.2s-dw4 or conformer-small or 16L-16s-overlapped" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/tests.log | sed 's/ *\[.*%\]//' | tail -80
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
for v in a nofwd3 b; do
  case $v in nofwd3) E="KDFM_ATTN_FWD3=0" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_$v.log 2>&1 || { tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
exit $rc
