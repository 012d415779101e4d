# round 6: fp8 unit tests (measured tolerance), fp8 kernel-only timing, XL step kernel trace (bf16)
set -o pipefail
OUT=gpurun_out/r6e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big_tests.log 2>&1
rc=$?
tail -3 $OUT/big_tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python3 -u tools/gemm_xl_micro.py > $OUT/xl.log 2>&1 || { echo "micro failed"; tail -5 $OUT/xl.log; exit 5; }
cat $OUT/xl.log | tr '|' '\n' | grep -E "M=|fp8|fwd big "
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o xl --output-format csv -- python3 -u tools/xl_step.py 2 bf16 > $OUT/xl_prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/xl_prof.log; exit 6; }
echo prof ok
exit $rc
