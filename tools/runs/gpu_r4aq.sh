# hardware queues per process: default (4) vs 8, interleaved bench
set -o pipefail
OUT=gpurun_out/r4aq
mkdir -p $OUT
export TMPDIR=/tmp
v() { tail -1 $1 | cut -c1-140 | grep -o '"value": [0-9.]*'; }
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_q4_$r.log 2>&1 || { echo "bench failed"; exit 7; }
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_q8_$r.log 2>&1 || { echo "bench q8 failed"; exit 8; }
  echo "q4 $(v $OUT/bench_q4_$r.log)  q8 $(v $OUT/bench_q8_$r.log)"
done
