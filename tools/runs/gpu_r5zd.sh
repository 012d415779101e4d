# kv_prep split over (kind, head) tile groups: attention tests, then the bench at 1 / 2 / all tiles per workgroup
set -o pipefail
OUT=gpurun_out/r5zd
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attn_fwd3_gpu.py tests/test_step_parity_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
for hpw in 1 2 8 1 2 8; do
  KDFM_KVPREP_HPW=$hpw timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/b$hpw.log 2>&1 || { echo "bench failed"; tail -5 $OUT/b$hpw.log; exit 3; }
  echo "hpw=$hpw $(tail -1 $OUT/b$hpw.log | cut -c1-100)"
done
exit $rc
