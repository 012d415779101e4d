# kernel trace of the bench step on the round's tree: summary, timeline, the compute stream's kernel sequence
set -o pipefail
OUT=gpurun_out/r6aq
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; tail $OUT/prof_bench.log; exit 4; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 8 200 > $OUT/kernel_summary.txt
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv > $OUT/timeline.txt
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv seq > $OUT/seq.txt
gzip -c $OUT/prof/run_kernel_trace.csv > $OUT/kernel_trace.csv.gz
rm -rf $OUT/prof
tail -1 $OUT/seq.txt; head -8 $OUT/timeline.txt
