# round-4 measurement pass: bench line, rocprofv3 kernel trace of the bench, PMC traffic (separate passes)
set -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
bash tools/pmc_traffic.sh r4k_pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 5; }
echo "pmc ok"
