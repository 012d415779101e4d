# bwd2 dQ staging through buffer loads (no spills): attention backward tests, phase probe, micro
set -o pipefail
OUT=gpurun_out/r4ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attn_bwd_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 3; }
tail -2 $OUT/tests.log
timeout -k 10 120 ./tools/attn_bwd_probe > $OUT/probe.log 2>&1 || { echo "probe failed"; exit 4; }
grep -E "us per launch|probe (1|2|3|4|5|6|30|31):" $OUT/probe.log
timeout -k 10 200 python -u tools/attn_bwd2_micro.py 20 > $OUT/micro.log 2>&1 || { echo "micro failed"; exit 5; }
cat $OUT/micro.log
