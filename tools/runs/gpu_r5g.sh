# isolated attention forward timings (prepared-operand fwd3 at student / teacher shapes, dropout on/off)
set -o pipefail
OUT=gpurun_out/r5g
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/attn3_micro.py > $OUT/attn3.log 2>&1 || { echo "attn3 micro failed"; tail -5 $OUT/attn3.log; exit 3; }
cat $OUT/attn3.log
