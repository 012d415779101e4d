# BN-SiLU backward reduce with 8 loads in flight, 8-accumulator LN fold: tests, bench x2
set -o pipefail
OUT=gpurun_out/r6ad
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_ffn_gpu.py tests/test_lnproj_gpu.py tests/test_determinism_gpu.py tests/test_step_parity_gpu.py tests/test_bench_shape_gpu.py > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { echo bench failed; exit 3; }
  tail -1 $OUT/bench.log | grep -o '"value": [0-9.]*'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || exit 4
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 8 200 > $OUT/kernel_summary.txt
rm -rf $OUT/prof
grep -E "bn_silu_bwd_reduce|ln_fold" $OUT/kernel_summary.txt
