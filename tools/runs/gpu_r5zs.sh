# decoder weight gradient on the weight-gradient stream (KDFM_DEC_SIDE=1) vs in line on the compute stream, where
# the r5final2 trace shows it (wgr 113 us + scalar fold 152 us) right before the encoder backward: bench A/B
set -o pipefail
OUT=gpurun_out/r5zs
mkdir -p $OUT
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_DEC_SIDE=1
  run KDFM_DEC_SIDE=0
done
