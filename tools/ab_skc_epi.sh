#!/bin/bash
# A/B of the skc compile-time epilogues (KDFM_SKC_FAST_EPI=1, default) against the generic one (=0):
# kernel scan + full-step bench for each, after the bf16 kernel tests.
set -o pipefail
OUT=gpurun_out/ab_epi
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_skinny_gpu.py tests/test_kernels_gpu.py tests/test_ddp_overlap_gpu.py tests/test_rowstream_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for f in 0 1; do
  KDFM_SKC_FAST_EPI=$f timeout -k 10 120 python -u tools/skc_scan.py > $OUT/scan_$f.log 2>&1 || exit 1
  KDFM_SKC_FAST_EPI=$f timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$f.log 2>&1 || exit 1
  echo "fast=$f: $(grep -E ' 205312 | 821248 ' $OUT/scan_$f.log | cut -c1-90 | tr '\n' ' ')"
  echo "fast=$f: $(tail -1 $OUT/bench_$f.log | cut -c100-160)"
done
