# round-6 closing measurement (5: the round's last tree): full GPU suite, the default bench line, a kernel trace of the bench (summary,
# timeline, roofline agreement), PMC traffic and MFMA passes
set -o pipefail
OUT=gpurun_out/r6final5
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1
rc=$?
tail -1 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 700 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 8 200 > $OUT/kernel_summary.txt
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv > $OUT/timeline.txt
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv gaps > $OUT/gaps.txt 2>&1 || true
python3 tools/roofline_check.py $OUT/prof_bench.log $OUT/prof/run_kernel_trace.csv > $OUT/roofline_check.txt
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv
rm -rf $OUT/prof
echo "prof ok"
bash tools/pmc_traffic.sh r6final5_pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 5; }
echo "pmc ok"
bash tools/pmc_mfma.sh r6final5_mfma > $OUT/mfma.log 2>&1 || { echo "mfma failed"; tail -5 $OUT/mfma.log; exit 6; }
echo "mfma ok"
exit $rc
