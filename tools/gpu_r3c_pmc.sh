#!/bin/bash
# round 3: SQ counters of the fused kernels in isolation (tools/ffn_micro.py, tools/attn_bwd_micro.py) and
# of the bench step (tools/pmc_mfma.sh): MFMA busy, wait / stall / active shares of the wave cycles
set -o pipefail
OUT=gpurun_out/r3c
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in 1 2; do
  if [ $pass = 1 ]; then C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAVES"; else
    C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/ffn_p$pass" -o run \
    -- python3 -u tools/ffn_micro.py 10 > "$OUT/ffn_p$pass.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/attn_p$pass" -o run \
    -- python3 -u tools/attn_bwd_micro.py 10 0.1 > "$OUT/attn_p$pass.log" 2>&1 || exit $?
done
mkdir -p "$OUT/ffn" "$OUT/attn"
mv "$OUT/ffn_p1" "$OUT/ffn/p1" && mv "$OUT/ffn_p2" "$OUT/ffn/p2" && mv "$OUT/attn_p1" "$OUT/attn/p1" && mv "$OUT/attn_p2" "$OUT/attn/p2"
python3 tools/pmc_mfma.py "$OUT/ffn" > "$OUT/ffn_mfma.txt" 2>&1
python3 tools/pmc_mfma.py "$OUT/attn" > "$OUT/attn_mfma.txt" 2>&1
bash tools/pmc_mfma.sh r3c/step > "$OUT/step_mfma.log" 2>&1 || exit $?
echo done
