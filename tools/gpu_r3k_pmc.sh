#!/bin/bash
# round 3: SQ instruction / wait counters of the subsampling conv2 data-gradient kernel variants
set -o pipefail
OUT=gpurun_out/r3k/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
P3="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
i=0
for C in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/p$i" -o run \
    -- python3 -u tools/ss_dgrad_probe.py > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 tools/pmc_dump.py "$OUT" ss_dgrad > "$OUT/ss_dgrad_pmc.txt" 2>&1
echo done
