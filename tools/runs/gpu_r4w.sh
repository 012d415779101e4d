set -o pipefail
OUT=gpurun_out/r4w
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a decmain w192 w384 b decmain2 w128; do
  case $v in decmain*) E="KDFM_DEC_SIDE=0" ;; w192) E="KDFM_WGR_WGS=192" ;; w384) E="KDFM_WGR_WGS=384" ;; w128) E="KDFM_WGR_WGS=128" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
