# the DDP bitwise-equivalence check repeated in one process (its intermittent failure, with diagnostics)
set -o pipefail
OUT=gpurun_out/r5zz
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/ddp_equiv_repeat.py 6 > $OUT/ddp.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/ddp.log | cut -c1-400 | tail -14
exit $rc
