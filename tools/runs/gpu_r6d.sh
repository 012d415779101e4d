# round 6: biggemm (bf16 + fp8) tests, big-vs-generic step diagnostic, big-route / fp8 XL step parity, micro + tile sweep,
# XL step timing
set -o pipefail
OUT=gpurun_out/r6d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big_tests.log 2>&1
rc=$?
tail -3 $OUT/big_tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python3 -u tools/big_step_diag.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail -5 $OUT/diag.log; exit 3; }
cat $OUT/diag.log
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py -k "big_route or fp8" > $OUT/step.log 2>&1
rc2=$?
grep -E "PASS|FAIL|rel err" $OUT/step.log | head -80
[ $rc2 -le 1 ] || exit 4
timeout -k 10 300 python3 -u tools/gemm_xl_micro.py > $OUT/xl.log 2>&1 || { echo "micro failed"; tail -5 $OUT/xl.log; exit 5; }
cat $OUT/xl.log
timeout -k 10 300 python3 -u tools/xl_step.py 3 bf16 > $OUT/xl_step.log 2>&1 || { echo "xl step failed"; tail -5 $OUT/xl_step.log; exit 6; }
cat $OUT/xl_step.log
timeout -k 10 300 python3 -u tools/xl_step.py 3 fp8 > $OUT/xl_step8.log 2>&1 || { echo "xl fp8 step failed"; tail -5 $OUT/xl_step8.log; exit 7; }
cat $OUT/xl_step8.log
exit $((rc + rc2))
