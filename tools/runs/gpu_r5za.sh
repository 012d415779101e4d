# isolated subsampling kernels (fused forward student / teacher, dgrad)
set -o pipefail
OUT=gpurun_out/r5za
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/ss_micro.py > $OUT/ss.log 2>&1 || { echo "ss micro failed"; tail -5 $OUT/ss.log; exit 3; }
cat $OUT/ss.log
