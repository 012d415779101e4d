# heads-backward half order A/B + kernel trace of the new default
set -o pipefail
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_determinism_gpu.py tests/test_race_gpu.py tests/test_plan_gpu.py tests/test_ddp_overlap_gpu.py tests/test_bench_shape_gpu.py > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; grep -E "FAILED" $OUT/tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in after before after2 before2; do
  case $v in after*) E="KDFM_HEADS_BWD_ORDER=after" ;; before*) E="KDFM_HEADS_BWD_ORDER=before" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
