#!/bin/bash
# three-way A/B (current / dQ-only / previous library), then per-kernel durations of current vs previous
set -o pipefail
OUT=gpurun_out/r3ac
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in all dq prev; do
    L=""; [ $lib != all ] && L=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_$lib.so
    KDFM_LIB=$L timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${lib}_$rep.log" 2>&1 || exit 1
    echo "$lib rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${lib}_$rep.log | head -1)"
  done
done
for lib in all prev; do
  L=""; [ $lib != all ] && L=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_$lib.so
  export KDFM_LIB=$L
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$lib" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > "$OUT/prof_$lib.log" 2>&1 || exit 1
done
unset KDFM_LIB
