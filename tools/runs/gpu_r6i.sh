#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6i
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/fp8_big_debug.py > gpurun_out/r6i/dbg.log 2>&1; echo "dbg exit $?"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_biggemm_gpu.py > gpurun_out/r6i/big.log 2>&1 || { echo big failed; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py -k "fp8 or big_route" > gpurun_out/r6i/step.log 2>&1 || { echo step failed; exit 1; }
timeout -k 10 200 python tools/xl_step.py 3 fp8 > gpurun_out/r6i/xl_fp8.log 2>&1
timeout -k 10 200 python tools/gemm_xl_micro.py > gpurun_out/r6i/micro.log 2>&1
