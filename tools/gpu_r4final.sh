# round-4 closing measurement: the default bench line, a kernel trace of the bench, PMC traffic and MFMA passes
set -o pipefail
OUT=gpurun_out/r4final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; exit 4; }
echo "prof ok"
bash tools/pmc_traffic.sh r4final_pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 5; }
echo "pmc ok"
bash tools/pmc_mfma.sh r4final_mfma > $OUT/mfma.log 2>&1 || { echo "mfma failed"; tail -5 $OUT/mfma.log; exit 6; }
echo "mfma ok"
