#!/bin/bash
# bench A/B over the row-parallel wgrad knobs (output-row slices KDFM_WGR_MSL, workgroup target
# KDFM_WGR_WGS), two rounds each on one box
set -o pipefail
OUT=gpurun_out/${1:-envab}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "1 0" "0 0" "1 256" "0 256"; do
    set -- $cfg
    KDFM_WGR_MSL=$1 KDFM_WGR_WGS=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_$1_$2_$rep.log 2>&1 || exit 3
    echo "MSL=$1 WGS=$2 rep=$rep $(tail -1 $OUT/b_$1_$2_$rep.log | cut -c90-150)"
  done
done
