#!/bin/bash
# bench at several row-parallel wgrad workgroup targets (KDFM_WGR_WGS), two rounds on one box
set -o pipefail
OUT=gpurun_out/${1:-wgsb}
mkdir -p $OUT
for rep in 1 2; do
  for w in 128 192 256; do
    KDFM_WGR_WGS=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${w}_$rep.log 2>&1 || exit 3
    echo "WGS=$w rep=$rep $(tail -1 $OUT/b_${w}_$rep.log | cut -c90-150)"
  done
done
