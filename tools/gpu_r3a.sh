#!/bin/bash
# round 3: attention LSE-recompute kernels, wide-vocab losses, the race checker and the overlapped-
# schedule tests
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attn_bwd_gpu.py \
  tests/test_attn_fused_gpu.py tests/test_ctc_gpu.py > gpurun_out/r3a/attn_tests.log 2>&1
rc=$?
echo "attn tests rc=$rc" >> gpurun_out/r3a/attn_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/attn_bwd_micro.py 20 0.1 > gpurun_out/r3a/attn_micro.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/race_check.py --layers 3 --batch 8 > gpurun_out/r3a/race_ddp.log 2>&1
rc=$?
echo "race rc=$rc" >> gpurun_out/r3a/race_ddp.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_determinism_gpu.py \
  tests/test_ddp_overlap_gpu.py tests/test_plan_gpu.py > gpurun_out/r3a/overlap_tests.log 2>&1
echo "overlap tests rc=$?" >> gpurun_out/r3a/overlap_tests.log
