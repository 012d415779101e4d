set -o pipefail
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a noepi noload b; do
  case $v in noepi) E="KDFM_BN_EPI=0" ;; noload) E="KDFM_BN_ON_LOAD=0" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
