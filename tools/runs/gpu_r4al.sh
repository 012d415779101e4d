# BN-SiLU backward reduce: >= 192-row chunks, at most 64 per channel group (was 201 x 64-row chunks): tests, step A/B + chunk sweep
set -o pipefail
OUT=gpurun_out/r4al
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bn or dwconv" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -1 $OUT/tests.log
v() { tail -1 $1 | cut -c1-140 | grep -o '"value": [0-9.]*'; }
for r in 1 2; do
  KDFM_LIB=$PWD/ab/libkdfm_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_base$r.log 2>&1 || { echo "bench base failed"; exit 7; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_new$r.log 2>&1 || { echo "bench new failed"; exit 8; }
  KDFM_BNRED_CHUNKS=24 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_c24_$r.log 2>&1 || { echo "bench c24 failed"; exit 9; }
  KDFM_BNRED_CHUNKS=128 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_c128_$r.log 2>&1 || { echo "bench c128 failed"; exit 9; }
  echo "base $(v $OUT/bench_base$r.log)  new(64) $(v $OUT/bench_new$r.log)  c24 $(v $OUT/bench_c24_$r.log)  c128 $(v $OUT/bench_c128_$r.log)"
done
