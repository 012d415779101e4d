#!/bin/bash
# One GPU-box pass: gpu tests, bench, rocprofv3 kernel stats.  Every GPU step has its own time
# limit and the steps are chained with && so the first failure ends the call.
# usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag> [tests|notests]
set -o pipefail
TAG=${1:-run}
MODE=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step_tests() {
  [ "$MODE" = "tests" ] || return 0
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
}
step_bench() {
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.log" 2>&1
}
step_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
}
step_tests && echo "tests ok" && step_bench && echo "bench ok" && tail -1 "$OUT/bench.log" && step_prof && echo "prof ok"
rc=$?
tail -3 "$OUT/pytest_gpu.log" 2>/dev/null
exit $rc
