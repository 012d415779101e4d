set -o pipefail
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_subsample_gpu.py tests/test_attn_bwd_gpu.py tests/test_nemo_api_gpu.py tests/test_race_gpu.py tests/test_training_rng_gpu.py tests/test_ddp_overlap_nondet_gpu.py tests/test_optim_gpu.py tests/test_determinism_gpu.py tests/test_step_parity_gpu.py tests/test_bench_shape_gpu.py > gpurun_out/r4b/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4b/tests.log
grep -E "FAILED|ERROR" gpurun_out/r4b/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-sensitivity"
for v in new old cus64 cus128 new2; do
  case $v in
    new|new2) E="" ;;
    old) E="KDFM_SS_ONE_KERNEL=0 KDFM_ATTN_BWD2=0" ;;
    cus64) E="KDFM_WGRAD_CUS=64" ;;
    cus128) E="KDFM_WGRAD_CUS=128" ;;
  esac
  env $E timeout -k 10 200 $B > gpurun_out/r4b/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r4b/bench_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r4b/bench_$v.log | cut -c1-160)"
done
timeout -k 10 200 python -u tools/plan_issue_probe.py 6 40 > gpurun_out/r4b/plan_issue.log 2>&1
tail -45 gpurun_out/r4b/plan_issue.log
