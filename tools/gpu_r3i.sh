#!/bin/bash
# round 3: frontend FFT kernel (16 waves, pipelined frame loads), NoiseAdapter backward (16 lanes per row,
# ordered partial fold), the adapter's dx route; parity of the touched kernels, then the bench + profile
set -o pipefail
OUT=gpurun_out/r3i
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/frontend_micro.py 20 > "$OUT/frontend_micro.log" 2>&1 || exit $?
timeout -k 10 120 python -u tools/route_probe.py > "$OUT/route_probe.log" 2>&1 || exit $?
timeout -k 10 120 python -u tools/ss_dgrad_probe.py > "$OUT/ss_dgrad_probe.log" 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_step_parity_gpu.py::test_frontend_matches_oracle" tests/test_heads_golden_gpu.py \
  tests/test_heads_versions_gpu.py "tests/test_step_parity_gpu.py::test_ver5_step_matches_oracle[2L-1.2s]" \
  tests/test_determinism_gpu.py tests/test_nemo_api_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity \
  > "$OUT/bench.log" 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > "$OUT/prof_bench.log" 2>&1 || exit $?
f=$(find "$OUT/prof" -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 8 > "$OUT/kernel_summary.txt" 2>&1
python3 tools/timeline.py "$f" > "$OUT/timeline.txt" 2>&1
echo done
