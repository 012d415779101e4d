# same-box A/B: BN-SiLU reduce / LN fold changes (current) vs HEAD's convmod.hip + norm.hip (ab/libkdfm_base.so)
set -o pipefail
OUT=gpurun_out/r6ae
mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed $1"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*' | head -1)"
}
for r in 1 2 3; do
  run KDFM_X=new
  run KDFM_LIB=ab/libkdfm_base.so
done
