# which kdfm_gemm (non-large-tile) launches the XL step issues
set -o pipefail
OUT=gpurun_out/r6o
mkdir -p $OUT
timeout -k 10 300 python tools/gemm_calls.py $OUT/xl_gemm_calls.txt xl > $OUT/run.log 2>&1; echo "rc $?"
