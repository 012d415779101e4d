#!/bin/bash
# round 3 measurement pass: attention probe, full GPU suite, bench, kernel-trace profile, PMC HBM traffic
set -o pipefail
mkdir -p gpurun_out/r3f2
timeout -k 10 120 ./tools/attn_probe > gpurun_out/r3f2/attn_probe.log 2>&1 || exit 1
grep -E "relpos|probe  1:|probe 31:" gpurun_out/r3f2/attn_probe.log
bash tools/gpu_full.sh r3f2 || exit $?
f=$(find gpurun_out/r3f2/prof -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 5 > gpurun_out/r3f2/kernel_summary.txt 2>&1
python3 tools/timeline.py "$f" > gpurun_out/r3f2/timeline.txt 2>&1
bash tools/pmc_traffic.sh r3f2_pmc || exit $?
