# A/B: teacher stream at high priority
set -o pipefail
OUT=gpurun_out/r5zb
mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity"
for cfg in "KDFM_X=0" "KDFM_TEACHER_PRIO=1" "KDFM_X=0" "KDFM_TEACHER_PRIO=1"; do
  env $cfg timeout -k 10 200 $B > $OUT/b.log 2>&1 || { echo "bench failed [$cfg]"; tail -5 $OUT/b.log; exit 3; }
  echo "[$cfg] $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
