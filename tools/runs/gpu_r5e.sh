# head-dim-128 tests (valid-square comparison), then the r5d kernel-trace profile of the current tree
set -o pipefail
OUT=gpurun_out/r5e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attn_bwd_gpu.py -k head_dim > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
bash tools/runs/gpu_r5d.sh || exit 4
exit $rc
