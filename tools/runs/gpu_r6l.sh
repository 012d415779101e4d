# XL sensitivity order check; XL fp8 step kernel mix
set -o pipefail
OUT=gpurun_out/r6l
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python tools/xl_sens.py > $OUT/xl_sens.log 2>&1; echo "sens $?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/xl_step.py 3 fp8 > $OUT/xl_prof.log 2>&1 || { echo prof failed; exit 1; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 3 40 > $OUT/xl_fp8_kernel_summary.txt 2>&1
rm -rf $OUT/prof
