#!/bin/bash
# bench A/B: stream priorities off / on (KDFM_STREAM_PRIO), after the wgrad tests
set -o pipefail
OUT=gpurun_out/${1:-prio}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py tests/test_fm_chain_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 180 python -u tools/wgrad_micro.py > $OUT/micro.log 2>&1 && grep bf16 $OUT/micro.log
for p in 0 1 0 1; do
  KDFM_STREAM_PRIO=$p timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$p.log 2>&1 || exit 3
  echo "prio=$p $(tail -1 $OUT/bench_$p.log | cut -c90-200)"
done
