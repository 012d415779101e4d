#!/bin/bash
# A measurement pass on the GPU box: tools/gpu_full.sh (the -m gpu suite, the bench, a rocprofv3 kernel
# trace of a bench run), then the per-step kernel summary and the stream timeline with the compute
# stream's gaps attributed to their producers.  usage (repo root, via gpurun): bash tools/gpu_pass.sh <tag> [notests]
set -o pipefail
T=${1:-pass}
OUT=gpurun_out/$T
mkdir -p "$OUT"
if [ "$2" = "notests" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 3; }
  tail -1 "$OUT/bench.log" | cut -c1-400
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > "$OUT/prof_bench.log" 2>&1 || { echo "prof failed"; exit 4; }
else
  bash tools/gpu_full.sh "$T" || exit $?
fi
f=$(find "$OUT/prof" -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 0 60 > "$OUT/kernel_summary.txt" 2>&1
python3 tools/timeline.py "$f" gaps > "$OUT/timeline.txt" 2>&1
head -30 "$OUT/kernel_summary.txt"
head -20 "$OUT/timeline.txt"
