# A/B: weight-gradient stream CU mask (KDFM_WGRAD_CUS) 0 / 224 / 192, interleaved x2
set -o pipefail
OUT=gpurun_out/r6t
mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed $1"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_WGRAD_CUS=0
  run KDFM_WGRAD_CUS=224
  run KDFM_WGRAD_CUS=192
done
