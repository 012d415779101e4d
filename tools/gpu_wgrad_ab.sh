#!/bin/bash
# wgrad A/B on one box: the wgrad tests, the micro-benchmark with 4- vs 8-column bf16 staging units
# (KDFM_WGR_BIN8) and with / without output-row slices (KDFM_WGR_MSL), then the bench.
set -o pipefail
OUT=gpurun_out/${1:-wab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py tests/test_ffn_gpu.py tests/test_lnproj_gpu.py tests/test_fm_chain_gpu.py tests/test_denoise_chain_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
KDFM_WGR_BIN8=0 KDFM_WGR_MSL=0 timeout -k 10 180 python -u tools/wgrad_micro.py > $OUT/micro_base.log 2>&1 && grep -v amdgpu.ids $OUT/micro_base.log
timeout -k 10 180 python -u tools/wgrad_micro.py > $OUT/micro_new.log 2>&1 && grep -v amdgpu.ids $OUT/micro_new.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-260
