# conv0 flip diagnosis with the decoders seeded (seeds 0 / 1) and the seeded logit-KD module test
set -o pipefail
OUT=gpurun_out/r5zf
mkdir -p $OUT
for s in 0 1; do
  DIAG_SEED=$s timeout -k 10 200 python3 -u tools/conv0_diag.py > $OUT/diag_seed$s.log 2>&1 || { echo "diag failed"; tail -20 $OUT/diag_seed$s.log; exit 2; }
  grep -v amdgpu.ids $OUT/diag_seed$s.log
done
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_nemo_api_gpu.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
exit $rc
