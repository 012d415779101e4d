# CTC gradient kernel with parallel label lists, KL with one loss atomic per workgroup: tests, bench A/B against
# the previous loss.hip (ab/libkdfm_base.so), kernel trace
set -o pipefail
OUT=gpurun_out/r5zo
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ctc_gpu.py tests/test_step_parity_gpu.py tests/test_nemo_api_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_X=new
  run KDFM_LIB=ab/libkdfm_base.so
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 8 200 > $OUT/kernel_summary.txt && grep -i "total\|ctc\|kl_kernel" $OUT/kernel_summary.txt
exit $rc
