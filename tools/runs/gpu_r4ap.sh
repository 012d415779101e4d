# subsampling conv2 weight-gradient columns built early on the weight-gradient stream (KDFM_EARLY_COLS): step parity, A/B
set -o pipefail
OUT=gpurun_out/r4ap
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_step_parity_gpu.py tests/test_subsample_gpu.py tests/test_ddp_overlap_gpu.py tests/test_ddp_overlap_nondet_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -1 $OUT/tests.log
v() { tail -1 $1 | cut -c1-140 | grep -o '"value": [0-9.]*'; }
for r in 1 2 3; do
  KDFM_EARLY_COLS=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_off$r.log 2>&1 || { echo "bench off failed"; exit 7; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_on$r.log 2>&1 || { echo "bench on failed"; exit 8; }
  echo "off $(v $OUT/bench_off$r.log)  on $(v $OUT/bench_on$r.log)"
done
