set -o pipefail
OUT=gpurun_out/r4x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_wgrad_gpu.py tests/test_step_parity_gpu.py tests/test_determinism_gpu.py tests/test_bench_shape_gpu.py -k "not 16L" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; grep -E "FAILED" $OUT/tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a b; do
  timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
