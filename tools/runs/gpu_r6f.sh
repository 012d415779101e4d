# round 6: MX fp8 (probe, unit tests, XL step parity), per-step weight copies, LN backward for wide rows, dwconv K=9,
# the XL step timings and micro, XL/FC f32 step parity (dwconv K=9, LN paths)
set -o pipefail
OUT=gpurun_out/r6f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 python3 -u tools/fp8_probe.py > $OUT/fp8_probe.log 2>&1; echo "probe rc=$?"; grep -E "MATCH|per-lane|cvt" $OUT/fp8_probe.log
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big_tests.log 2>&1
rc=$?
tail -3 $OUT/big_tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_step_parity_gpu.py -k "big_route or fp8 or xl or fastconformer or large" > $OUT/step.log 2>&1
rc2=$?
grep -E "PASSED|FAILED|step losses|layer . output" $OUT/step.log | head -40
[ $rc2 -le 1 ] || exit 4
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_lnproj_gpu.py > $OUT/kern.log 2>&1
rc3=$?
tail -2 $OUT/kern.log
[ $rc3 -le 1 ] || exit 5
timeout -k 10 300 python3 -u tools/xl_step.py 3 bf16 > $OUT/xl_step.log 2>&1 || { echo "xl step failed"; tail -5 $OUT/xl_step.log; exit 6; }
cat $OUT/xl_step.log
timeout -k 10 300 python3 -u tools/xl_step.py 3 fp8 > $OUT/xl_step8.log 2>&1 || { echo "xl fp8 step failed"; tail -5 $OUT/xl_step8.log; exit 7; }
cat $OUT/xl_step8.log
timeout -k 10 300 python3 -u tools/gemm_xl_micro.py > $OUT/xl.log 2>&1 || { echo "micro failed"; tail -5 $OUT/xl.log; exit 8; }
cat $OUT/xl.log | tr '|' '\n' | grep -E "M=|fp8"
exit $((rc + rc2 + rc3))
