#!/bin/bash
# Waves-per-workgroup sweep of the LDS-slab conv kernel (results: profiles/r01_sweep/).  Variant
# libraries are built beforehand on the CPU, e.g. for WV in 4 12:
#   hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -DKDFM_SKC_WV=$WV -c csrc/skinny.hip \
#     -o build_exp/skinny_wv$WV.o && hipcc -shared --offload-arch=gfx950 -o kdfm/libkdfm_wv$WV.so \
#     <csrc/build/*.o except skinny.o> build_exp/skinny_wv$WV.o
# and selected per run with KDFM_LIB (kdfm/_lib.py).
set -o pipefail
mkdir -p gpurun_out/sweep
for v in default wv4 wv12; do
  if [ $v = default ]; then L=""; else L="$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_$v.so"; fi
  KDFM_LIB=$L timeout -k 10 120 python -u tools/skc_scan.py > gpurun_out/sweep/scan_$v.log 2>&1 || exit 1
  KDFM_LIB=$L timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sweep/bench_$v.log 2>&1 || exit 1
  echo "$v: $(grep 205312 gpurun_out/sweep/scan_$v.log)"
  echo "$v: $(tail -1 gpurun_out/sweep/bench_$v.log | cut -c100-175)"
done
