# round 6: biggemm tests (fixed size floor), big-vs-generic step diagnostic, fp8 MFMA lane-map probe, tile-shape sweep
set -o pipefail
OUT=gpurun_out/r6c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big_tests.log 2>&1
rc=$?
tail -3 $OUT/big_tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 60 python3 -u tools/fp8_probe.py > $OUT/fp8_probe.log 2>&1; echo "fp8 probe rc=$?"; cat $OUT/fp8_probe.log
timeout -k 10 300 python3 -u tools/big_step_diag.py > $OUT/diag.log 2>&1 || { echo "diag failed"; tail -5 $OUT/diag.log; exit 3; }
cat $OUT/diag.log
for t in 0 1 2; do
  KDFM_BIG_TILE=$t timeout -k 10 300 python3 -u tools/gemm_xl_micro.py > $OUT/xl_tile$t.log 2>&1 || { echo "micro failed"; tail -5 $OUT/xl_tile$t.log; exit 4; }
  echo "tile $t"; cut -c1-330 $OUT/xl_tile$t.log
done
exit $rc
