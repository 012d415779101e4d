# 3-stage LDS ring in the large-tile GEMM: tests, micro NS=3 vs 2, XL steps NS=3 vs 2
set -o pipefail
OUT=gpurun_out/r6ai
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_biggemm_gpu.py > $OUT/big.log 2>&1 || { echo big failed; tail -30 $OUT/big.log; exit 1; }
tail -1 $OUT/big.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_step_parity_gpu.py -k "big_route or fp8 or 1024 or 512" > $OUT/step.log 2>&1 || { echo step failed; tail -30 $OUT/step.log; exit 1; }
tail -1 $OUT/step.log
for ns in 3 2; do
  KDFM_BIG_NS=$ns timeout -k 10 200 python tools/gemm_xl_micro.py > $OUT/micro_ns$ns.log 2>&1 || exit 1
done
for ns in 3 2 3 2; do
  KDFM_BIG_NS=$ns timeout -k 10 200 python tools/xl_step.py 3 bf16 > $OUT/xl.log 2>&1 || exit 1
  echo "NS=$ns $(tail -1 $OUT/xl.log | cut -c1-40)"
done
