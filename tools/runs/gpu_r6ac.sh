# A/B: student bf16 mirror (KDFM_BF16_MIRROR) on the XL bf16 step, interleaved
set -o pipefail
OUT=gpurun_out/r6ac
mkdir -p $OUT
for r in 1 2; do
  for m in 0 1; do
    KDFM_BF16_MIRROR=$m timeout -k 10 200 python tools/xl_step.py 4 bf16 > $OUT/run.log 2>&1 || exit 1
    echo "mirror=$m $(tail -2 $OUT/run.log | cut -c1-40 | tr '\n' ' ')"
  done
done
