#!/bin/bash
# round 3: FFN backward with 4 chunk parities per row tile; step plans under the recorded reduction
# mode; then the bench and a kernel profile of the step
set -o pipefail
OUT=gpurun_out/r3f
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ffn_gpu.py "tests/test_step_parity_gpu.py::test_frontend_matches_oracle" \
  tests/test_plan_gpu.py tests/test_determinism_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/ffn_micro.py 20 > "$OUT/ffn_micro.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity \
  > "$OUT/bench.log" 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > "$OUT/prof_bench.log" 2>&1 || exit $?
f=$(find "$OUT/prof" -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 8 > "$OUT/kernel_summary.txt" 2>&1
python3 tools/timeline.py "$f" > "$OUT/timeline.txt" 2>&1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_encfm_gpu.py \
  > "$OUT/encfm_tests.log" 2>&1
echo "encfm tests rc=$?" >> "$OUT/encfm_tests.log"
echo done
