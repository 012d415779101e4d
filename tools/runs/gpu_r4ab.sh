# attention backward v2 micro: dQ alone and beside a weight-gradient burst; kernel trace of the same
set -o pipefail
OUT=gpurun_out/r4ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/attn_bwd2_micro.py 20 > $OUT/micro.log 2>&1 || { echo "micro failed"; tail -20 $OUT/micro.log; exit 3; }
cat $OUT/micro.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 -u tools/attn_bwd2_micro.py 10 > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
