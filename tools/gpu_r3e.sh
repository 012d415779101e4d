#!/bin/bash
# round 3: bench (plan replay, with the bounded all-core CPU baseline) on the p~ attention backward,
# eager bench, step / optimizer / DDP tests, then the SQ counters of the fused kernels
set -o pipefail
OUT=gpurun_out/r3e
mkdir -p "$OUT"
python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))" > "$OUT/host.txt"
cat /sys/fs/cgroup/cpu.max >> "$OUT/host.txt" 2>&1
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --eager --no-f32-sensitivity --no-cpu-baseline \
  > "$OUT/bench_eager.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py \
  tests/test_optim_gpu.py tests/test_ddp_overlap_gpu.py tests/test_ddp_equiv_gpu.py tests/test_plan_gpu.py \
  > "$OUT/step_tests.log" 2>&1
echo "step tests rc=$?" >> "$OUT/step_tests.log"
bash tools/gpu_r3c_pmc.sh > "$OUT/pmc.log" 2>&1
echo "pmc rc=$?" >> "$OUT/pmc.log"
