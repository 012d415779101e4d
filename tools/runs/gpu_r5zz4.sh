# DDP equivalence repeats with the heads' first layer half NOT split onto its own stream (KDFM_HEADS_SPLIT=0)
set -o pipefail
OUT=gpurun_out/r5zz4
mkdir -p $OUT
KDFM_HEADS_SPLIT=0 timeout -k 10 500 python3 -u tools/ddp_equiv_repeat.py 8 > $OUT/ddp.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/ddp.log | grep "MISMATCH\|mismatching" | cut -c1-200
exit $rc
