set -o pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_wgrad_gpu.py tests/test_determinism_gpu.py tests/test_bench_shape_gpu.py tests/test_race_gpu.py tests/test_plan_gpu.py tests/test_ddp_overlap_gpu.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; grep -E "FAILED" $OUT/tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in new nopair nofold4 new2 nopair2; do
  case $v in new|new2) E="KDFM_WGR_FOLD4=1" ;; nopair|nopair2) E="KDFM_WGRAD_PAIRS=0" ;; nofold4) E="KDFM_WGR_FOLD4=0 KDFM_WGRAD_PAIRS=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c1-140)"
done
