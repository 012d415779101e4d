#!/bin/bash
# wgrad micro-benchmark at several workgroup targets (KDFM_WGR_WGS) and min 32-row steps per split
set -o pipefail
OUT=gpurun_out/${1:-wgs}
mkdir -p $OUT
for cfg in "256 4" "512 4" "768 4" "512 2"; do
  set -- $cfg
  KDFM_WGR_WGS=$1 KDFM_WGR_STEPS=$2 timeout -k 10 180 python -u tools/wgrad_micro.py > $OUT/micro_$1_$2.log 2>&1 || exit 1
  echo "== WGS=$1 STEPS=$2"; grep -v amdgpu.ids $OUT/micro_$1_$2.log
done
