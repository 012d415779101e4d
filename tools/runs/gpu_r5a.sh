# round 5 first GPU pass: head-dim-128 attention kernels vs float64, the meta-encoder workspace test,
# then the bench line on this tree
set -o pipefail
OUT=gpurun_out/r5a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_attn_bwd_gpu.py \
  tests/test_attn_fused_gpu.py "tests/test_encfm_meta_gpu.py::test_meta_workspace_follows_batch_shape" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-400
exit $rc
