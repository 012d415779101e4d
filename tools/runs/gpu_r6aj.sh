# XCD-grouped column slices in the row-parallel weight gradient: bitwise tests, s2conv micro, bench A/B
set -o pipefail
OUT=gpurun_out/r6aj
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py tests/test_subsample_gpu.py > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python tools/s2conv_micro.py > $OUT/micro.log 2>&1 || { cat $OUT/micro.log; exit 1; }
cat $OUT/micro.log
for f in 0 1 0 1; do
  KDFM_WGR_XGRP=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_$f.log 2>&1 || { tail -20 $OUT/bench_$f.log; exit 1; }
  echo "XGRP=$f $(grep -o '"value": [0-9.]*' $OUT/bench_$f.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$f.log | head -1)"
done
