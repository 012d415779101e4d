# frozen-teacher bf16 twins / fragment images cached by FlatStore.version (no per-step rebuild): the GPU suite's
# engine / checkpoint / module / parity tests (the whole GPU suite), bench A/B (KDFM_TEACHER_CACHE 1 / 0)
set -o pipefail
OUT=gpurun_out/r5zr
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
for i in 1 0 1 0; do
  KDFM_TEACHER_CACHE=$i timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b$i.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$i.log; exit 3; }
  echo "cache=$i $(tail -1 $OUT/b$i.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
done
exit $rc
