set -o pipefail
OUT=gpurun_out/r4aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a f1 b f2 c f3; do
  case $v in f*) E="KDFM_FFT_GRID=256" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-170)"
done
