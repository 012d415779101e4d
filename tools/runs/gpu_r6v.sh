set -o pipefail
OUT=gpurun_out/r6v
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/xl_cmp.py fp8 keep > $OUT/cmp_fp8_shared_streams.log 2>&1; echo "rc $?"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_plan_gpu.py tests/test_determinism_gpu.py tests/test_ddp_equiv_gpu.py tests/test_ddp_overlap_gpu.py tests/test_rccl_gpu.py tests/test_race_gpu.py > $OUT/tests.log 2>&1; echo "tests $?"; tail -1 $OUT/tests.log
