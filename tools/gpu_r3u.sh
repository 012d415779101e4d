#!/bin/bash
# round 3: kernel-argument placement experiment (HIP_FORCE_DEV_KERNARG), interleaved bench A/B
set -o pipefail
OUT=gpurun_out/r3u
mkdir -p "$OUT"
for rep in 1 2; do
  for kv in 1 0; do
    HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${kv}_$rep.log" 2>&1 || exit 1
    echo "kernarg=$kv rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${kv}_$rep.log | head -1)"
  done
done
