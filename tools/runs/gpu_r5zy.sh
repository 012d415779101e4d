# the LDS-DMA weight-gradient kernel's split depth (KDFM_WGD_STEPS: row steps per split of the KD heads' long
# reductions; default 12): bench A/B 8 / 12 / 24
set -o pipefail
OUT=gpurun_out/r5zy
mkdir -p $OUT
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_WGD_STEPS=12
  run KDFM_WGD_STEPS=8
  run KDFM_WGD_STEPS=24
done
