# weight-gradient workgroup target for the conv-mode (denoiser) products only: 256 (default) vs 128 / 64, interleaved
set -o pipefail
OUT=gpurun_out/r4an${R4AN_SUFFIX}
mkdir -p $OUT
export TMPDIR=/tmp
v() { tail -1 $1 | cut -c1-140 | grep -o '"value": [0-9.]*'; }
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_256_$r.log 2>&1 || { echo "bench failed"; exit 7; }
  KDFM_WGR_CONV_WGS=384 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_384_$r.log 2>&1 || { echo "bench failed"; exit 7; }
  KDFM_WGR_CONV_WGS=512 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_512_$r.log 2>&1 || { echo "bench failed"; exit 7; }
  echo "256 $(v $OUT/bench_256_$r.log)  384 $(v $OUT/bench_384_$r.log)  512 $(v $OUT/bench_512_$r.log)"
done
