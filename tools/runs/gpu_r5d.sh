# round 5 profile of the current tree: rocprofv3 kernel trace of a short bench (summaries made on the CPU side)
set -o pipefail
OUT=gpurun_out/r5d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof_bench.log; exit 4; }
tail -1 $OUT/prof_bench.log | cut -c1-200
find $OUT/prof -name "*kernel_trace.csv" | head -3
