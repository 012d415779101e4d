# channel-pair depthwise forward + backward (d <= 128 default): kernel tests, micro, bench A/B
set -o pipefail
OUT=gpurun_out/r6am
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python tools/dwconv_micro.py 20 > $OUT/micro.log 2>&1 || { cat $OUT/micro.log; exit 1; }
cat $OUT/micro.log
for f in 0 1 0 1; do
  KDFM_DWC_P2=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_$f.log 2>&1 || { tail -20 $OUT/bench_$f.log; exit 1; }
  echo "P2=$f $(grep -o '"value": [0-9.]*' $OUT/bench_$f.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$f.log | head -1)"
done
