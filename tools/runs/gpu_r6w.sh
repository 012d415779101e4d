# bf16 producers for large-tile operands (dropout / BN-SiLU / GLU bwd), one weight epoch per train step
set -o pipefail
OUT=gpurun_out/r6w
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bf16_outputs_gpu.py tests/test_kernels_gpu.py > $OUT/unit.log 2>&1 || { echo unit failed; tail -30 $OUT/unit.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py tests/test_plan_gpu.py tests/test_determinism_gpu.py > $OUT/step.log 2>&1 || { echo step failed; tail -30 $OUT/step.log; exit 1; }
timeout -k 10 200 python tools/xl_step.py 3 bf16 > $OUT/xl_bf16.log 2>&1
timeout -k 10 200 python tools/xl_step.py 3 fp8 > $OUT/xl_fp8.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { echo bench failed; exit 3; }
tail -1 $OUT/bench.log | cut -c1-200
