#!/bin/bash
# One GPU-box pass: the whole -m gpu suite (no -x: every failure is reported), then, unless the test
# process died (fault / abort / timeout: rc other than 0 or 1), the bench and a rocprofv3 kernel trace.
# usage (from the repo root, via gpurun): bash tools/gpu_full.sh <tag>
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "test process rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 3; }
tail -1 "$OUT/bench.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > "$OUT/prof_bench.log" 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
exit $rc
