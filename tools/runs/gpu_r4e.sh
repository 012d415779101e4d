set -o pipefail
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ss_diag.py > gpurun_out/r4e/ss_diag.log 2>&1; echo "ss_diag rc=$?"; head -70 gpurun_out/r4e/ss_diag.log
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_race_gpu.py tests/test_nemo_api_gpu.py tests/test_step_parity_gpu.py -k "race or logit or fastconformer" > gpurun_out/r4e/tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed|Error|bad|RACE|err " gpurun_out/r4e/tests.log | head -40
