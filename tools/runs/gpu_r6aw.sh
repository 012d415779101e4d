# the frozen teacher's weight twins / images rebuilt on the teacher stream (KDFM_TEACHER_PREP_SIDE): GPU suite, bench A/B
set -o pipefail
OUT=gpurun_out/r6aw
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1
rc=$?
tail -1 $OUT/tests.log
[ $rc -le 1 ] || exit 2
for rep in 1 2 3; do
  for v in 0 1; do
    KDFM_TEACHER_PREP_SIDE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_tp${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_tp${v}_$rep.log; exit 4; }
    echo "tprep=$v rep $rep: $(grep -o '"value": [0-9.]*' $OUT/bench_tp${v}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_tp${v}_$rep.log | head -1) $(grep -o 'step plan ([0-9]* recorded' $OUT/bench_tp${v}_$rep.log | head -1)"
  done
done
exit $rc
