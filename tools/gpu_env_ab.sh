#!/bin/bash
# interleaved step A/B of one environment setting against the default (same library, same box)
# usage: tools/gpu_env_ab.sh NAME=VALUE [reps]
set -o pipefail
OUT=gpurun_out/env_ab
mkdir -p "$OUT"
SET="$1"; REPS=${2:-3}
for rep in $(seq 1 $REPS); do
  for arm in env base; do
    if [ $arm = env ]; then
      env "$SET" timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${arm}_$rep.log" 2>&1 || exit 1
    else
      timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${arm}_$rep.log" 2>&1 || exit 1
    fi
    echo "$arm($SET) rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${arm}_$rep.log | head -1)"
  done
done
