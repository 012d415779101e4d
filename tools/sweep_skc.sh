set -o pipefail
mkdir -p gpurun_out/sweep
for v in default wv4 wv12; do
  if [ $v = default ]; then L=""; else L="$PWD/kd-via-fm-in-asr_amd/kdfm/libkdfm_$v.so"; fi
  KDFM_LIB=$L timeout -k 10 120 python -u tools/skc_scan.py > gpurun_out/sweep/scan_$v.log 2>&1 || exit 1
  KDFM_LIB=$L timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sweep/bench_$v.log 2>&1 || exit 1
  echo "$v: $(grep 205312 gpurun_out/sweep/scan_$v.log)"
  echo "$v: $(tail -1 gpurun_out/sweep/bench_$v.log | cut -c100-175)"
done
