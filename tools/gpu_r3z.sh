#!/bin/bash
# attention prologue fragment loads: attention tests + step parity, probe, library A/B on one box
set -o pipefail
OUT=gpurun_out/r3z
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_fused_gpu.py \
  tests/test_attn_bwd_gpu.py tests/test_step_parity_gpu.py tests/test_determinism_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
bash tools/gpu_r3w.sh
