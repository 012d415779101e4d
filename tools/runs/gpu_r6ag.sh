# 16-byte-lane elementwise kernels (qkv prep, GLU fwd/bwd, BN-SiLU fwd, dropout): tests, XL timing, headline
set -o pipefail
OUT=gpurun_out/r6ag
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bf16_outputs_gpu.py tests/test_kernels_gpu.py tests/test_training_rng_gpu.py tests/test_step_parity_gpu.py tests/test_determinism_gpu.py tests/test_bench_shape_gpu.py tests/test_versions_gpu.py > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python tools/xl_step.py 3 bf16 > $OUT/xl_bf16.log 2>&1
timeout -k 10 200 python tools/xl_step.py 3 fp8 > $OUT/xl_fp8.log 2>&1
tail -1 $OUT/xl_bf16.log; tail -1 $OUT/xl_fp8.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { echo bench failed; exit 3; }
tail -1 $OUT/bench.log | grep -o '"value": [0-9.]*' | head -1
