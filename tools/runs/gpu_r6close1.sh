# round-6 first closing measurement: full GPU suite, default bench line, kernel trace of the bench with its
# per-stream timeline and the roofline agreement check (tools/roofline_check.py)
set -o pipefail
OUT=gpurun_out/r6close1
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1
rc=$?
tail -1 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 8 200 > $OUT/kernel_summary.txt
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv > $OUT/timeline.txt
python3 tools/roofline_check.py $OUT/prof_bench.log $OUT/prof/run_kernel_trace.csv > $OUT/roofline_check.txt
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv
rm -rf $OUT/prof
echo "prof ok"
exit $rc
