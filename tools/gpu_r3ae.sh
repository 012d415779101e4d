#!/bin/bash
# depthwise-conv round: micro-benchmark (previous / current library), kernel GPU tests, step A/B
set -o pipefail
OUT=gpurun_out/r3ae
mkdir -p "$OUT"
KDFM_LIB=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_prev.so timeout -k 10 200 python -u tools/dwconv_micro.py 50 > "$OUT/micro_prev.log" 2>&1 || exit 1
timeout -k 10 200 python -u tools/dwconv_micro.py 50 > "$OUT/micro_new.log" 2>&1 || exit 1
paste "$OUT/micro_prev.log" "$OUT/micro_new.log"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2 3; do
  for lib in new prev; do
    L=""; [ $lib = prev ] && L=$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_prev.so
    KDFM_LIB=$L timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > "$OUT/bench_${lib}_$rep.log" 2>&1 || exit 1
    echo "$lib rep=$rep $(grep -o '"value": [0-9.]*' $OUT/bench_${lib}_$rep.log | head -1)"
  done
done
