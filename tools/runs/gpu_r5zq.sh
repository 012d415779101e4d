# workgroup target of the subsampling conv2 weight-gradient gather (KDFM_WGR_C2D_WGS 256 / 512 / 768): bench A/B
set -o pipefail
OUT=gpurun_out/r5zq
mkdir -p $OUT
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_WGR_C2D_WGS=256
  run KDFM_WGR_C2D_WGS=512
  run KDFM_WGR_C2D_WGS=768
done
