# round-5 second closing measurement (after the late-round changes): full GPU suite, the default bench line, a
# kernel trace of the bench, PMC traffic and MFMA passes
set -o pipefail
OUT=gpurun_out/r5final2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests > $OUT/tests.log 2>&1
rc=$?
tail -1 $OUT/tests.log
# an assertion failure (rc 1) is read afterwards; a crash / hang ends the call
[ $rc -le 1 ] || exit 2
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
bash tools/pmc_traffic.sh r5final2_pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 5; }
echo "pmc ok"
bash tools/pmc_mfma.sh r5final2_mfma > $OUT/mfma.log 2>&1 || { echo "mfma failed"; tail -5 $OUT/mfma.log; exit 6; }
echo "mfma ok"
