# isolated FFN fused-kernel timings (student / teacher shapes)
set -o pipefail
OUT=gpurun_out/r5z
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/ffn_micro.py > $OUT/ffn.log 2>&1 || { echo "ffn micro failed"; tail -5 $OUT/ffn.log; exit 3; }
cat $OUT/ffn.log
