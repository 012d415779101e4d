# isolated weight-gradient products at several split targets (KDFM_WGR_WGS): per-step rate vs partial traffic
set -o pipefail
OUT=gpurun_out/r5w
mkdir -p $OUT
for w in 256 128 64 32; do
  echo "== KDFM_WGR_WGS=$w"
  KDFM_WGR_WGS=$w timeout -k 10 200 python3 -u tools/wgrad_micro.py > $OUT/w$w.log 2>&1 || { echo "micro failed"; tail -5 $OUT/w$w.log; exit 3; }
  grep "bf16 ffn\|bf16 qkv\|bf16 out" $OUT/w$w.log
done
