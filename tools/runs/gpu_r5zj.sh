# FM chain with register B operands (permlane32 swaps instead of LDS staging) + weight-gradient split depth 6:
# FM chain / wgrad / heads / step-parity tests, bench x2, kernel trace
set -o pipefail
OUT=gpurun_out/r5zj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fm_chain_gpu.py tests/test_wgrad_gpu.py tests/test_heads_golden_gpu.py tests/test_heads_versions_gpu.py tests/test_step_parity_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b$i.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$i.log; exit 3; }
  echo "$(tail -1 $OUT/b$i.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 8 40 > $OUT/kernel_summary.txt && grep -i "total\|fm_chain\|wgr" $OUT/kernel_summary.txt
exit $rc
