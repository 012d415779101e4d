# padded y1 rows + LDS-staged y2 epilogue in the fused subsampling forward: GPU suite, isolated micro (y1
# unpadded / padded), PMC write bytes of the micro, interleaved bench A/B (KDFM_SS_Y1_PAD=0 vs default)
set -o pipefail
OUT=gpurun_out/r6ap
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for ld in 88 96; do
  SS_Y1_LD=$ld timeout -k 10 120 python -u tools/ss_micro.py > $OUT/ss_micro_$ld.log 2>&1 || { tail -20 $OUT/ss_micro_$ld.log; exit 2; }
  echo "ld $ld:"; cat $OUT/ss_micro_$ld.log | grep -v amdgpu.ids | head -12
done
for ld in 88 96; do
  SS_Y1_LD=$ld timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/w$ld -o run \
    -- python3 -u tools/ss_micro.py > $OUT/pmc_w$ld.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc_w$ld.log; exit 3; }
  python3 - $OUT/w$ld <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "ss_fused" in k:
        print(sys.argv[1], k, "WRITE_SIZE avg KB", sum(v) / len(v), "n", len(v))
PY
  rm -rf $OUT/w$ld
done
for rep in 1 2 3; do
  for v in base pad; do
    case $v in base) P=0;; pad) P=1;; esac
    KDFM_SS_Y1_PAD=$P timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench_${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_${v}_$rep.log; exit 4; }
    echo "$v rep $rep: $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_$rep.log | head -1)"
  done
done
