#!/bin/bash
# round 3: bf16 weight gradients streamed by LDS-DMA (wgd_kernel): probe timing on/off, wgrad-consuming
# tests, bench on/off
set -o pipefail
OUT=gpurun_out/r3t
mkdir -p "$OUT"
timeout -k 10 120 ./tools/wgrad_probe > "$OUT/wgrad_probe_dma.log" 2>&1 || { tail -5 "$OUT/wgrad_probe_dma.log"; exit 1; }
KDFM_WGD=0 timeout -k 10 120 ./tools/wgrad_probe > "$OUT/wgrad_probe_old.log" 2>&1 || exit 1
grep "wgrad_bf16" "$OUT/wgrad_probe_dma.log" "$OUT/wgrad_probe_old.log"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_gpu.py \
  tests/test_encfm_gpu.py tests/test_heads_golden_gpu.py tests/test_fm_chain_gpu.py tests/test_determinism_gpu.py \
  tests/test_step_parity_gpu.py tests/test_ddp_overlap_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench.log" 2>&1 || exit $?
grep -o '"value": [0-9.]*' "$OUT/bench.log" | head -1
KDFM_WGD=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_old.log" 2>&1 || exit $?
grep -o '"value": [0-9.]*' "$OUT/bench_old.log" | head -1
