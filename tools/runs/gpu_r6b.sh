# round 6: the large-tile bf16 GEMM (csrc/biggemm.hip) -- its unit tests, the XL product micro vs hipBLASLt, the bf16
# step parity cases that route through it; the race checker's mutations; the bench line (plan-replay roofline)
set -o pipefail
OUT=gpurun_out/r6b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big_tests.log 2>&1
rc=$?
tail -3 $OUT/big_tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python3 -u tools/gemm_xl_micro.py > $OUT/xl.log 2>&1 || { echo "xl micro failed"; tail -5 $OUT/xl.log; exit 5; }
cat $OUT/xl.log
timeout -k 10 200 python3 -u tools/gemm_xl_micro.py large > $OUT/large.log 2>&1 || { echo "large micro failed"; tail -5 $OUT/large.log; exit 5; }
cat $OUT/large.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_race_gpu.py tests/test_step_parity_gpu.py -k "race or bf16 or checker or allreduce" > $OUT/tests.log 2>&1
rc2=$?
tail -3 $OUT/tests.log
[ $rc2 -le 1 ] || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 4; }
tail -1 $OUT/bench.log | cut -c1-600
exit $((rc + rc2))
