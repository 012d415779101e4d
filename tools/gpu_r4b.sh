set -o pipefail
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_race_gpu.py tests/test_training_rng_gpu.py tests/test_ddp_overlap_nondet_gpu.py tests/test_optim_gpu.py tests/test_determinism_gpu.py tests/test_step_parity_gpu.py > gpurun_out/r4b/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4b/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/plan_issue_probe.py 6 40 > gpurun_out/r4b/plan_issue.log 2>&1
cat gpurun_out/r4b/plan_issue.log | tail -45
