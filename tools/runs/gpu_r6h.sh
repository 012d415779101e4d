#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 120 python tools/fp8_scale_probe.py > gpurun_out/r6h/scale_probe.log 2>&1
echo "probe exit $?"
