# DDP equivalence repeats: with a host sync between the backward and the final bucket launches (diagnosis)
set -o pipefail
OUT=gpurun_out/r5zz2
mkdir -p $OUT
DDP_DIAG_SYNC=1 timeout -k 10 500 python3 -u tools/ddp_equiv_repeat.py 6 > $OUT/ddp.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/ddp.log | grep "run \|mismatching" | cut -c1-260
exit $rc
