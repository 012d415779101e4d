# skinny kernel: compile-time MSE epilogue (the FM loss head leaves the generic, spilling instance): tests, trace, step A/B
set -o pipefail
OUT=gpurun_out/r4ak
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_skinny_gpu.py tests/test_gemm_gpu.py tests/test_heads_golden_gpu.py tests/test_heads_versions_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -1 $OUT/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 4; }
for r in 1 2 3; do
  KDFM_LIB=$PWD/ab/libkdfm_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_base$r.log 2>&1 || { echo "bench base failed"; exit 7; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_new$r.log 2>&1 || { echo "bench new failed"; exit 8; }
  echo "base $(tail -1 $OUT/bench_base$r.log | cut -c1-140 | grep -o '"value": [0-9.]*')  new $(tail -1 $OUT/bench_new$r.log | cut -c1-140 | grep -o '"value": [0-9.]*')"
done
