#!/bin/bash
# attention GPU tests on the current library, then an interleaved A/B against libkdfm_prev.so (3 reps)
set -o pipefail
OUT=gpurun_out/r3ad
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attn_bwd_gpu.py tests/test_attn_fused_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2 3; do
  for lib in new prev; do
    L=""; [ $lib = prev ] && L=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_prev.so
    KDFM_LIB=$L timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${lib}_$rep.log" 2>&1 || exit 1
    echo "$lib rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${lib}_$rep.log | head -1)"
  done
done
