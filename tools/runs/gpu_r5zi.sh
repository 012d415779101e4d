# A/B continued: split depth 6 / 12 / 16 and the workgroup target 192 at depth 6
set -o pipefail
OUT=gpurun_out/r5zi
mkdir -p $OUT
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_WGR_STEPS=6
  run KDFM_WGR_STEPS=12
  run KDFM_WGR_STEPS=16
  run "KDFM_WGR_STEPS=6 KDFM_WGR_WGS=192"
done
