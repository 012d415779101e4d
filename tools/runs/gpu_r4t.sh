set -o pipefail
OUT=gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ss_probe > $OUT/ss_probe.log 2>&1 || { echo "probe failed"; tail -3 $OUT/ss_probe.log; exit 3; }
timeout -k 10 200 python -u tools/ss_micro.py > $OUT/ss_micro.log 2>&1 || { echo "micro failed"; exit 3; }
grep -v amdgpu.ids $OUT/ss_micro.log
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; grep -E "FAILED" $OUT/tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a c192 b c224; do
  case $v in c192) E="KDFM_WGRAD_CUS=192" ;; c224) E="KDFM_WGRAD_CUS=224" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
