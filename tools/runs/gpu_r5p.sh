# in-step kernel profile of the current tree (kernel trace + timeline)
set -o pipefail
OUT=gpurun_out/r5p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof_bench.log; exit 4; }
tail -1 $OUT/prof_bench.log | cut -c1-200
