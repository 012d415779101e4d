# A/B with deferred folds in place: row-parallel weight-gradient split depth (KDFM_WGR_STEPS: at least N 32-row
# steps per split; 4 = ~100 splits of the 12 832-row products) -- fewer splits, fewer partial bytes
set -o pipefail
OUT=gpurun_out/r5zh
mkdir -p $OUT
for st in 4 8 6 4 8 6; do
  KDFM_WGR_STEPS=$st timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b$st.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$st.log; exit 3; }
  echo "steps=$st $(tail -1 $OUT/b$st.log | grep -o '"value": [0-9.]*, "unit": "utterances/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
done
