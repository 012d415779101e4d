# student bf16 mirror written by AdamW (wide models): tests, XL timing
set -o pipefail
OUT=gpurun_out/r6ab
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_optim_gpu.py tests/test_checkpoint.py > $OUT/unit.log 2>&1 || { echo unit failed; tail -30 $OUT/unit.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py -k "big_route or fp8 or 1024 or 512" > $OUT/step.log 2>&1 || { echo step failed; tail -30 $OUT/step.log; exit 1; }
timeout -k 10 200 python tools/xl_step.py 3 bf16 > $OUT/xl_bf16.log 2>&1
timeout -k 10 200 python tools/xl_step.py 3 fp8 > $OUT/xl_fp8.log 2>&1
