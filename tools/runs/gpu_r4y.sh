set -o pipefail
OUT=gpurun_out/r4y
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a pt b pt2; do
  case $v in pt*) E="KDFM_STREAM_PRIO=teacher" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
