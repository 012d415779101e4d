# stream schedule knobs on the round-6 tree: high-priority critical streams (KDFM_STREAM_PRIO=1), CTC/KL on a
# stream of its own (KDFM_AUX_STREAM=1), against the default; interleaved, 2 reps
set -o pipefail
OUT=gpurun_out/r6ak
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in base prio aux; do
    case $v in base) E="";; prio) E="KDFM_STREAM_PRIO=1";; aux) E="KDFM_AUX_STREAM=1";; esac
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_${v}_$rep.log; exit 1; }
    echo "$v rep $rep: $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1)"
  done
done
