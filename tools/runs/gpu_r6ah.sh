# XL bf16 step: kernel mix + per-stream timeline
set -o pipefail
OUT=gpurun_out/r6ah
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/xl_step.py 4 bf16 > $OUT/xl_prof.log 2>&1 || { echo prof failed; exit 1; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_trace.csv 4 60 > $OUT/xl_bf16_kernel_summary.txt 2>&1
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv > $OUT/xl_timeline.txt 2>&1
python3 tools/timeline.py $OUT/prof/run_kernel_trace.csv gaps > $OUT/xl_gaps.txt 2>&1 || true
rm -rf $OUT/prof
