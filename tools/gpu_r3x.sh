#!/bin/bash
# LN-block prologue restructure: kernel tests, FFN probe / micro, library A/B on one box
set -o pipefail
OUT=gpurun_out/r3x
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ffn_gpu.py tests/test_lnproj_gpu.py \
  tests/test_step_parity_gpu.py tests/test_determinism_gpu.py tests/test_bench_shape_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 120 ./tools/ffn_probe > "$OUT/ffn_probe.log" 2>&1 || exit 1
timeout -k 10 120 python tools/ffn_micro.py > "$OUT/ffn_micro.log" 2>&1 || exit 1
cat "$OUT/ffn_micro.log" | grep -v amdgpu.ids
bash tools/gpu_r3w.sh
