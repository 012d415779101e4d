# denoiser conv weight gradients issued at the end of each heads backward half (KDFM_DEFER_DENO_WG=1): parity, A/B
set -o pipefail
OUT=gpurun_out/r4as
mkdir -p $OUT
export TMPDIR=/tmp
KDFM_DEFER_DENO_WG=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_step_parity_gpu.py tests/test_heads_golden_gpu.py tests/test_heads_versions_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -1 $OUT/tests.log
v() { tail -1 $1 | cut -c1-140 | grep -o '"value": [0-9.]*'; }
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_off$r.log 2>&1 || { echo "bench off failed"; exit 7; }
  KDFM_DEFER_DENO_WG=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_on$r.log 2>&1 || { echo "bench on failed"; exit 8; }
  echo "off $(v $OUT/bench_off$r.log)  on $(v $OUT/bench_on$r.log)"
done
