# default re-check on the final tree: side-stream LN folds, deferred folds off, register-staged dQ, unpaired
# weight gradients -- each against the default, interleaved
set -o pipefail
OUT=gpurun_out/r5zw
mkdir -p $OUT
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_X=default
  run KDFM_SIDE_FOLDS=1
  run KDFM_FOLD_DEFER=0
  run KDFM_ATTN_DQ3=0
  run KDFM_WGRAD_PAIRS=0
done
