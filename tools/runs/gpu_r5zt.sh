# short reductions (< 64 row steps: the per-layer positional-projection weight gradients over 801 rows) split into
# 2-step chunks (KDFM_WGR_SHORT_STEPS 2 vs 0 = the general 6): wgrad tests, step parity, bench A/B
set -o pipefail
OUT=gpurun_out/r5zt
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_wgrad_gpu.py tests/test_step_parity_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_WGR_SHORT_STEPS=2
  run KDFM_WGR_SHORT_STEPS=0
done
exit $rc
