#!/bin/bash
# round 6: MX scale-slot probe, depthwise-striding forward rewrite tests, XL step timing
set -o pipefail
mkdir -p gpurun_out/r6g
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/fp8_probe.py > gpurun_out/r6g/probe.log 2>&1
echo "probe exit $?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_dw_striding_gpu.py tests/test_subsample_gpu.py > gpurun_out/r6g/dws.log 2>&1 || { echo dws failed; exit 1; }
timeout -k 10 200 python tools/xl_step.py 3 bf16 > gpurun_out/r6g/xl.log 2>&1
