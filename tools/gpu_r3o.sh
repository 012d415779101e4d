#!/bin/bash
# round 3: the ver5 heads in two layer halves (first half beside the encoders' second half / the encoder
# backward's first half): parity, determinism, plans, DDP, bench with and without the split
set -o pipefail
OUT=gpurun_out/r3o
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_step_parity_gpu.py tests/test_determinism_gpu.py tests/test_plan_gpu.py tests/test_heads_versions_gpu.py \
  tests/test_ddp_overlap_gpu.py tests/test_ddp_equiv_gpu.py tests/test_nemo_api_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity \
  > "$OUT/bench_split.log" 2>&1 || exit $?
KDFM_HEADS_SPLIT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity \
  > "$OUT/bench_nosplit.log" 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > "$OUT/prof_bench.log" 2>&1 || exit $?
f=$(find "$OUT/prof" -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 8 > "$OUT/kernel_summary.txt" 2>&1
python3 tools/timeline.py "$f" > "$OUT/timeline.txt" 2>&1
echo done
