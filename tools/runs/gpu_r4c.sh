set -o pipefail
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r4c/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4c/tests.log
grep -E "FAILED|ERROR|Error" gpurun_out/r4c/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in new xcd0 old cus64 new2; do
  case $v in
    new|new2) E="" ;;
    xcd0) E="KDFM_WGR_XCD=0" ;;
    old) E="KDFM_SS_ONE_KERNEL=0 KDFM_ATTN_BWD2=0 KDFM_WGR_XCD=0" ;;
    cus64) E="KDFM_WGRAD_CUS=64" ;;
  esac
  env $E timeout -k 10 200 $B > gpurun_out/r4c/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r4c/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r4c/bench_$v.log | cut -c1-160)"
done
