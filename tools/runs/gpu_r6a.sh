# round 6 first pass: the RCCL world-1 test, the extended race checker (serialised / plan / mutations), the
# deferred-fold and plan tests, DDP equivalence; bench line with the plan-replay roofline + a kernel trace of it
set -o pipefail
OUT=gpurun_out/r6a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_rccl_gpu.py tests/test_race_gpu.py \
  tests/test_wgrad_gpu.py tests/test_plan_gpu.py tests/test_ddp_equiv_gpu.py tests/test_ddp_overlap_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
timeout -k 10 200 python3 -u tools/gemm_xl_micro.py > $OUT/xl.log 2>&1 || { echo "xl micro failed"; tail -5 $OUT/xl.log; exit 5; }
cat $OUT/xl.log
exit $rc
