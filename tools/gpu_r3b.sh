#!/bin/bash
# round 3: DiffKD / V=1024 / overlapped-schedule parity, step plans, bench variants, kernel profile
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_diffkd_gpu.py \
  tests/test_plan_gpu.py "tests/test_step_parity_gpu.py" > gpurun_out/r3b/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3b/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/host_issue.py 5 > gpurun_out/r3b/host_issue.log 2>&1 || exit $?
for v in plan eager det; do
  case $v in
    plan) a="";;
    eager) a="--eager";;
    det) a="--deterministic";;
  esac
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-sensitivity $a \
    > gpurun_out/r3b/bench_$v.log 2>&1 || exit $?
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > gpurun_out/r3b/prof_bench.log 2>&1 || exit $?
f=$(find gpurun_out/r3b/prof -name '*kernel_trace.csv' -print -quit)
python3 tools/prof_summary.py "$f" 8 > gpurun_out/r3b/kernel_summary.txt 2>&1
python3 tools/timeline.py "$f" > gpurun_out/r3b/timeline.txt 2>&1
echo done
