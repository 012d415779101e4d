# bwd2 dQ: hoisted dropout key, branch-free dS elements: tests, probe, micro, step A/B
set -o pipefail
OUT=gpurun_out/r4aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attn_bwd_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -1 $OUT/tests.log
timeout -k 10 120 ./tools/attn_bwd_probe > $OUT/probe.log 2>&1 || { echo "probe failed"; exit 4; }
grep -E "us per launch|probe (1|2|5|6|30|31):" $OUT/probe.log
timeout -k 10 200 python -u tools/attn_bwd2_micro.py 20 > $OUT/micro.log 2>&1 || { echo "micro failed"; exit 5; }
head -3 $OUT/micro.log
for r in 1 2 3; do
  KDFM_LIB=$PWD/ab/libkdfm_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_base$r.log 2>&1 || { echo "bench base failed"; exit 7; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_new$r.log 2>&1 || { echo "bench new failed"; exit 8; }
  echo "base $(tail -1 $OUT/bench_base$r.log | cut -c1-140 | grep -o '"value": [0-9.]*')  new $(tail -1 $OUT/bench_new$r.log | cut -c1-140 | grep -o '"value": [0-9.]*')"
done
