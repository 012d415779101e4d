# row-tiled MX quantisation: fp8 tests, XL fp8 step parity and timing, micro
set -o pipefail
OUT=gpurun_out/r6m
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big.log 2>&1 || { echo big failed; tail -30 $OUT/big.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py -k "fp8" > $OUT/step.log 2>&1 || { echo step failed; exit 1; }
timeout -k 10 200 python tools/xl_step.py 3 fp8 > $OUT/xl_fp8.log 2>&1
timeout -k 10 200 python tools/gemm_xl_micro.py > $OUT/micro.log 2>&1
