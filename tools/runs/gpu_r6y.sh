# XL step kernel mix after the wide routing / LN / AdamW changes (bf16 and MX fp8)
set -o pipefail
OUT=gpurun_out/r6y
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for m in fp8 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run --output-format csv -- python3 tools/xl_step.py 3 $m > $OUT/xl_prof_$m.log 2>&1 || { echo prof failed; exit 1; }
  python3 tools/prof_summary.py $OUT/prof_$m/run_kernel_trace.csv 3 60 > $OUT/xl_${m}_kernel_summary.txt 2>&1
  rm -rf $OUT/prof_$m
done
