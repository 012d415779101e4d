# teacher FFN forward (d = 176) with 3 chunk parities per row tile (6 waves per workgroup, 1 203 waves instead
# of 802; residual rows loaded per piece, output over the accumulators): FFN tests, step parity, isolated micro
# and bench A/B against the previous ffn.hip (ab/libkdfm_base.so)
set -o pipefail
OUT=gpurun_out/r5zu
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ffn_gpu.py tests/test_step_parity_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 200 python3 -u tools/ffn_micro.py > $OUT/micro_new.log 2>&1 || { echo "micro failed"; tail -5 $OUT/micro_new.log; exit 3; }
KDFM_LIB=ab/libkdfm_base.so timeout -k 10 200 python3 -u tools/ffn_micro.py > $OUT/micro_base.log 2>&1 || { echo "micro failed"; exit 3; }
echo "new:"; cat $OUT/micro_new.log | tail -6; echo "base:"; cat $OUT/micro_base.log | tail -6
run() {
  env $1 timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/run.log 2>&1 || { echo "bench failed"; tail -5 $OUT/run.log; exit 3; }
  echo "$1 $(tail -1 $OUT/run.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
}
for r in 1 2; do
  run KDFM_X=new
  run KDFM_LIB=ab/libkdfm_base.so
done
exit $rc
