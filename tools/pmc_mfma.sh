#!/bin/bash
# Per-kernel MFMA busy and wave-state breakdown of the bench step from SQ counters (VERDICT r2 item 4:
# report MFMA busy next to TFLOP/s for the critical-path FFN / attention kernels).  One rocprofv3 --pmc
# pass per counter group (<= 8 SQ counters each), each under its own time limit; tools/pmc_mfma.py
# turns them into per-kernel MFMA-busy fractions (SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CU_CYCLES x 4
# SIMDs)) and wait / active shares of SQ_WAVE_CYCLES.
# usage (repo root, via gpurun): bash tools/pmc_mfma.sh <tag>
set -o pipefail
TAG=${1:-mfma}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAVES \
  --kernel-trace --output-format csv -d "$OUT/p1" -o run \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-sensitivity > "$OUT/p1.log" 2>&1 &&
echo "pass 1 ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  --kernel-trace --output-format csv -d "$OUT/p2" -o run \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-sensitivity > "$OUT/p2.log" 2>&1 &&
echo "pass 2 ok" &&
python3 tools/pmc_mfma.py "$OUT" > "$OUT/mfma.txt" && rm -rf "$OUT/p1" "$OUT/p2" && head -40 "$OUT/mfma.txt"
