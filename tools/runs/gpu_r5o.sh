# isolated weight-gradient products (wgrad_micro) and a kernel-trace of the same to split product vs fold
set -o pipefail
OUT=gpurun_out/r5o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/wgrad_micro.py > $OUT/wgrad.log 2>&1 || { echo "wgrad micro failed"; tail -5 $OUT/wgrad.log; exit 3; }
cat $OUT/wgrad.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u tools/wgrad_micro.py > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 4; }
