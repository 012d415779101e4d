# restructured attn_kv_prep (all heads per workgroup): fwd3 tests + step parity, then bench A/B of the
# wgrad split cap (KDFM_WGR_SMAX / KDFM_WGR_MSL) and the XL GEMM micro
set -o pipefail
OUT=gpurun_out/r5f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attn_fwd3_gpu.py tests/test_step_parity_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity"
for cfg in "" "KDFM_WGR_SMAX=32 KDFM_WGR_MSL=4" "KDFM_WGR_SMAX=24 KDFM_WGR_MSL=4" "KDFM_WGR_SMAX=48 KDFM_WGR_MSL=2" ""; do
  env $cfg timeout -k 10 200 $B > $OUT/b.log 2>&1 || { echo "bench failed [$cfg]"; tail -5 $OUT/b.log; exit 3; }
  echo "[$cfg] $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 200 python3 -u tools/gemm_xl_micro.py > $OUT/xl.log 2>&1 || { echo "xl micro failed"; tail -5 $OUT/xl.log; exit 5; }
cat $OUT/xl.log
exit $rc
