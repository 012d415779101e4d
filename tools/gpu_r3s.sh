#!/bin/bash
# round 3: attention forward with fixed-count p~ / m_blk buffer stores, FFN backward with the counted DMA
# barrier: probes, the kernels' tests, bench
set -o pipefail
OUT=gpurun_out/r3s
mkdir -p "$OUT"
timeout -k 10 120 ./tools/attn_probe > "$OUT/attn_probe.log" 2>&1 || exit $?
timeout -k 10 120 python tools/ffn_micro.py > "$OUT/ffn_micro.log" 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_fused_gpu.py \
  tests/test_attn_bwd_gpu.py tests/test_ffn_gpu.py tests/test_lnproj_gpu.py tests/test_determinism_gpu.py \
  tests/test_step_parity_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench.log" 2>&1 || exit $?
grep -o '"value": [0-9.]*' "$OUT/bench.log" | head -1
cat "$OUT/ffn_micro.log"
grep -E "relpos|probe (2|3|4|5|6|30|31):" "$OUT/attn_probe.log"
