# PMC breakdown of the fwd3 attention forward (teacher shape, dropout 0.1), isolated
set -o pipefail
OUT=${OUT:-gpurun_out/r5i}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
P="python3 -u tools/attn3_micro.py --pmc"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  --kernel-trace --output-format csv -d $OUT/p1 -o run -- $P > $OUT/p1.log 2>&1 && echo p1 ok &&
timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA \
  --kernel-trace --output-format csv -d $OUT/p2 -o run -- $P > $OUT/p2.log 2>&1 && echo p2 ok &&
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES \
  --kernel-trace --output-format csv -d $OUT/p3 -o run -- $P > $OUT/p3.log 2>&1 && echo p3 ok
exit 0
