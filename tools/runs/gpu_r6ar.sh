# cross-stream link events with a device-scope release (KDFM_LINK_EVENTS): event micro, GPU tests that exercise the
# schedule under the switch, interleaved bench A/B
set -o pipefail
OUT=gpurun_out/r6ar
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/event_micro.py > $OUT/event_micro.log 2>&1 || { tail -20 $OUT/event_micro.log; exit 1; }
grep -v amdgpu.ids $OUT/event_micro.log
for rep in 1 2; do
  for v in system device nofence; do
    KDFM_LINK_EVENTS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_${v}_$rep.log; exit 2; }
    echo "$v rep $rep: $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1)"
  done
done
KDFM_LINK_EVENTS=device timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_plan_gpu.py tests/test_race_gpu.py tests/test_determinism_gpu.py tests/test_rccl_gpu.py tests/test_bench_shape_gpu.py \
  tests/test_step_parity_gpu.py > $OUT/tests_device.log 2>&1 || { tail -30 $OUT/tests_device.log; exit 3; }
tail -1 $OUT/tests_device.log
