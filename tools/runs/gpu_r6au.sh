# teacher stream alone high-priority (KDFM_STREAM_PRIO=side: the teacher chain bounds the forward, the compute
# stream waits ~0.2 ms for it at the heads), and teacher + CTC/KL stream, against the default
set -o pipefail
OUT=gpurun_out/r6au
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in base side sideaux; do
    case $v in base) P=0;; side) P=side;; sideaux) P=side,aux;; esac
    KDFM_STREAM_PRIO=$P timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_${v}_$rep.log; exit 1; }
    echo "$v rep $rep: $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1)"
  done
done
