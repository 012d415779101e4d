#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6j
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/fp8_big_debug.py > gpurun_out/r6j/dbg.log 2>&1; echo "dbg exit $?"
