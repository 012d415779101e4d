# link events without the system fence by default: full GPU suite, the step plan's op list, bench lines
set -o pipefail
OUT=gpurun_out/r6as
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 200 python -u tools/plan_dump.py $OUT/plan_ops.txt > $OUT/plan_dump.log 2>&1 || { tail $OUT/plan_dump.log; exit 3; }
for rep in 1 2; do
  for v in system nofence; do
    KDFM_LINK_EVENTS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_${v}_$rep.log; exit 4; }
    echo "$v rep $rep: $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1)"
  done
done
exit $rc
