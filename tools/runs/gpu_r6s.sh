# multi-tile MX quantisation: tests, isolated timing at three grid caps, XL fp8 timing
set -o pipefail
OUT=gpurun_out/r6s
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_biggemm_gpu.py -k fp8 > $OUT/big.log 2>&1 || { echo big failed; tail -30 $OUT/big.log; exit 1; }
for c in 512 2048 1000000; do
  echo "cap $c" >> $OUT/quant.log
  KDFM_MXQ_GRID=$c timeout -k 10 120 python tools/quant_micro.py >> $OUT/quant.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/xl_step.py 3 fp8 > $OUT/xl_fp8.log 2>&1
