#!/bin/bash
# attention-backward round: phase probes (previous / current dQ kernel), attention GPU tests, then an
# interleaved A/B of the current library against libkdfm_prev.so
set -o pipefail
OUT=gpurun_out/r3ab
mkdir -p "$OUT"
timeout -k 10 120 ./tools/attn_bwd_probe_old > "$OUT/probe_old.log" 2>&1 || exit 1
timeout -k 10 120 ./tools/attn_bwd_probe > "$OUT/probe_new.log" 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attn_bwd_gpu.py tests/test_attn_fused_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
  for lib in new prev; do
    L=""; [ $lib = prev ] && L=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_prev.so
    KDFM_LIB=$L timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${lib}_$rep.log" 2>&1 || exit 1
    echo "$lib rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${lib}_$rep.log | head -1)"
  done
done
