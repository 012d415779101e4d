# bf16 dy2 from the subsampling output Linear's backward (kdfm_ss_out_dgrad) read by both conv2 gradients:
# subsample tests, step parity, bench, kernel profile
set -o pipefail
OUT=gpurun_out/r5r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_subsample_gpu.py tests/test_step_parity_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b.log; exit 3; }
  tail -1 $OUT/b.log | cut -c1-120
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
exit $rc
