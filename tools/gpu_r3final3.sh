#!/bin/bash
# round 3 closing pass: full GPU suite + bench + kernel trace (tools/gpu_full.sh), an interleaved A/B
# of the batched pos projection (KDFM_POS_BATCH=0 arm = per-layer), then the PMC HBM traffic passes
set -o pipefail
T=r3f3
bash tools/gpu_full.sh $T || exit $?
f=$(find gpurun_out/$T/prof -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/$T/kernel_summary.txt 2>&1
python3 tools/timeline.py "$f" > gpurun_out/$T/timeline.txt 2>&1
./tools/gpu_env_ab.sh KDFM_POS_BATCH=0 3 || exit $?
bash tools/pmc_traffic.sh ${T}_pmc || exit $?
