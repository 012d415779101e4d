set -o pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T -m gpu tests > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cm in 0 3 10; do
  KCM=$cm timeout -k 10 120 python -u tools/attn_small_diag.py > $OUT/attn_diag_cm$cm.log 2>&1 || { echo "diag failed"; tail -5 $OUT/attn_diag_cm$cm.log; exit 3; }
done
cat $OUT/attn_diag_cm3.log
B="python -u bench.py --steps 15 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in new; do
  case $v in new|new2) E="KDFM_WGR_FOLD4=1" ;; nopair|nopair2) E="KDFM_WGRAD_PAIRS=0" ;; nofold4) E="KDFM_WGR_FOLD4=0 KDFM_WGRAD_PAIRS=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c1-140)"
done
