#!/bin/bash
# A/B of two library builds on one box (KDFM_LIB), interleaved bench runs
set -o pipefail
OUT=gpurun_out/r3w
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in new prev; do
    L=""; [ $lib = prev ] && L=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_prev.so
    KDFM_LIB=$L timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${lib}_$rep.log" 2>&1 || exit 1
    echo "$lib rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${lib}_$rep.log | head -1)"
  done
done
