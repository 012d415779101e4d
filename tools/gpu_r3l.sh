#!/bin/bash
# round 3: subsampling conv2 data gradient rewrite (class-templated taps, per-wave decoded positions and
# mel patches in LDS, buffer addressing), BN / dwconv fold fusions; then the whole suite + bench + trace
set -o pipefail
OUT=gpurun_out/r3l
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/ss_dgrad_probe.py > "$OUT/ss_dgrad_probe.log" 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_subsample_gpu.py \
  > "$OUT/subsample_tests.log" 2>&1 || exit $?
bash tools/gpu_full.sh r3l/full
