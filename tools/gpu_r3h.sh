#!/bin/bash
# round 3: frontend kernel times (grid variants), the teacher's share of the critical path
set -o pipefail
OUT=gpurun_out/r3h
mkdir -p "$OUT"
for g in 2048 512 8192; do
  KDFM_FFT_GRID=$g timeout -k 10 120 python -u tools/frontend_micro.py 20 > "$OUT/frontend_g$g.log" 2>&1 || exit $?
done
timeout -k 10 400 python -u tools/teacher_ahead_probe.py 10 > "$OUT/teacher_probe.log" 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_plan_gpu.py tests/test_optim_gpu.py "tests/test_step_parity_gpu.py::test_ver5_step_matches_oracle[2L-1.2s-equal-widths]" \
  > "$OUT/plan.log" 2>&1
echo "plan rc=$?" >> "$OUT/plan.log"
