# ss_dgrad: tap loads pinned ahead of the mask loads, unconditional mel patch loads (no spills): tests, micro, step A/B
set -o pipefail
OUT=gpurun_out/r4ae
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_subsample_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -1 $OUT/tests.log
timeout -k 10 200 python -u tools/ss_micro.py > $OUT/ss_micro.log 2>&1 || { echo "ss micro failed"; exit 6; }
KDFM_LIB=$PWD/ab/libkdfm_base.so timeout -k 10 200 python -u tools/ss_micro.py > $OUT/ss_micro_base.log 2>&1 || { echo "ss micro base failed"; exit 6; }
echo "new: $(tail -1 $OUT/ss_micro.log)"; echo "base: $(tail -1 $OUT/ss_micro_base.log)"
for r in 1 2 3; do
  KDFM_LIB=$PWD/ab/libkdfm_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_base$r.log 2>&1 || { echo "bench base failed"; exit 7; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_new$r.log 2>&1 || { echo "bench new failed"; exit 8; }
  echo "base $(tail -1 $OUT/bench_base$r.log | cut -c1-140 | grep -o '"value": [0-9.]*')  new $(tail -1 $OUT/bench_new$r.log | cut -c1-140 | grep -o '"value": [0-9.]*')"
done
