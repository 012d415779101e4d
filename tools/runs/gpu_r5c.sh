# round 5 third pass: unet fold cropping fix, head-dim-128 test padding fix, XL sensitivity tolerance,
# then the XL sensitivity and a default bench
set -o pipefail
OUT=gpurun_out/r5c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attn_fwd3_gpu.py \
  tests/test_attn_bwd_gpu.py tests/test_encfm_meta_gpu.py \
  tests/test_step_parity_gpu.py -k "prepared or head_dim or meta or unet or xl" > $OUT/tests.log 2>&1
rc=$?
grep -E "(PASSED|FAILED|ERROR)" $OUT/tests.log | sed 's/ *\[.*%\]//' | tail -60
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit 2
timeout -k 10 600 python -u - > $OUT/xl_sens.log 2>&1 <<'PY'
import sys, json, torch
sys.path.insert(0, "."); sys.path.insert(0, "kd-via-fm-in-asr_amd")
import kdfm, bench
from kdfm import kernels as K
K.set_math("bf16")
r = bench.sensitivity(torch.device("cuda", 0), 256000, **bench.XL_SHAPES)
print(json.dumps(r))
PY
rc2=$?
tail -2 $OUT/xl_sens.log
exit $rc
