# deferred weight-gradient folds (one batched fold launch per Conformer layer): wgrad tests, step parity + DDP /
# race tests, bench A/B, kernel profile
set -o pipefail
OUT=gpurun_out/r5v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_wgrad_gpu.py tests/test_step_parity_gpu.py tests/test_race_gpu.py tests/test_ddp_overlap_nondet_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity"
for cfg in "KDFM_X=0" "KDFM_FOLD_DEFER=0" "KDFM_X=0" "KDFM_FOLD_DEFER=0"; do
  env $cfg timeout -k 10 200 $B > $OUT/b.log 2>&1 || { echo "bench failed [$cfg]"; tail -5 $OUT/b.log; exit 3; }
  echo "[$cfg] $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
exit $rc
