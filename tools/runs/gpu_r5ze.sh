# logit-KD module conv0 weight-gradient error vs the float64 oracle: deferred folds on / off
set -o pipefail
OUT=gpurun_out/r5ze
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/conv0_diag.py > $OUT/diag_defer1.log 2>&1 || { echo "diag failed"; tail -20 $OUT/diag_defer1.log; exit 2; }
cat $OUT/diag_defer1.log
KDFM_FOLD_DEFER=0 timeout -k 10 200 python3 -u tools/conv0_diag.py > $OUT/diag_defer0.log 2>&1 || { echo "diag failed"; tail -20 $OUT/diag_defer0.log; exit 2; }
cat $OUT/diag_defer0.log
