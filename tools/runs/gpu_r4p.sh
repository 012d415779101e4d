set -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/plan_dump.py $OUT/plan_after.txt > $OUT/dump.log 2>&1 || { tail -5 $OUT/dump.log; exit 3; }
KDFM_HEADS_BWD_ORDER=before timeout -k 10 200 python -u tools/plan_dump.py $OUT/plan_before.txt >> $OUT/dump.log 2>&1 || { tail -5 $OUT/dump.log; exit 3; }
wc -l $OUT/plan_*.txt
