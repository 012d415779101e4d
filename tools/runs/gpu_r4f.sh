set -o pipefail
mkdir -p gpurun_out/r4f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_encfm_meta_gpu.py tests/test_subsample_gpu.py tests/test_dw_striding_gpu.py tests/test_nemo_api_gpu.py tests/test_race_gpu.py tests/test_step_parity_gpu.py -k "meta or one_kernel or module_matches or logit or race or fastconformer" > gpurun_out/r4f/tests.log 2>&1; echo "tests rc=$?"
grep -E "PASSED|FAILED|worst|Error|bad|err " gpurun_out/r4f/tests.log | head -60
