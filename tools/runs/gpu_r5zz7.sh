# heads first half joins the teacher stream in the serialised schedule too (split restored there): DDP repeats, whole GPU suite, bench
# bench line (the overlapped schedule, unchanged)
set -o pipefail
OUT=gpurun_out/r5zz7
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/ddp_equiv_repeat.py 8 > $OUT/ddp.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/ddp.log | grep "MISMATCH\|mismatching" | cut -c1-200
[ $rc -le 1 ] || exit 2
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests > $OUT/tests.log 2>&1
rc2=$?
tail -3 $OUT/tests.log
[ $rc2 -le 1 ] || exit 3
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b.log; exit 4; }
tail -1 $OUT/b.log | cut -c1-160
exit $rc2
