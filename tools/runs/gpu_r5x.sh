# host issue of the recorded step plan vs the step (is the replay host-bound?)
set -o pipefail
OUT=gpurun_out/r5x
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/plan_issue_probe.py > $OUT/issue.log 2>&1 || { echo "probe failed"; tail -5 $OUT/issue.log; exit 3; }
tail -15 $OUT/issue.log
