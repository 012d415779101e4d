set -o pipefail
OUT=gpurun_out/r4z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_attn_fused_gpu.py tests/test_attn_bwd_gpu.py > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 2; }
tail -1 $OUT/tests.log
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in a sk256 sk1024 fft256 b; do
  case $v in sk256) E="KDFM_SKINNY_WGS=256" ;; sk1024) E="KDFM_SKINNY_WGS=1024" ;; fft256) E="KDFM_FFT_GRID=256" ;; fft1024) E="KDFM_FFT_GRID=1024" ;; *) E="KDFM_NONE=0" ;; esac
  env $E timeout -k 10 200 $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 $OUT/bench_$v.log | cut -c90-200)"
done
