#!/bin/bash
# round 3: teacher-graph determinism probe (where does the student mel differ), parity after the
# teacher auto-encoder moved to the teacher stream and the 16-lane adapter forward, per-call census,
# bench, SQ counters of the subsampling conv2 data gradient
set -o pipefail
OUT=gpurun_out/r3k
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/det_probe.py > "$OUT/det_probe.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_heads_golden_gpu.py tests/test_heads_versions_gpu.py tests/test_step_parity_gpu.py \
  tests/test_determinism_gpu.py tests/test_plan_gpu.py tests/test_nemo_api_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/census.py 60 > "$OUT/census.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity \
  > "$OUT/bench.log" 2>&1 || exit $?
bash tools/gpu_r3k_pmc.sh || exit $?
echo done
