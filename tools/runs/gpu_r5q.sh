# A/B: conv-mode weight-gradient workgroup target and a CU-masked weight-gradient stream (the 1.1 ms
# stream-1 gap before fm_chain_bwd behind the denoiser conv wgrads)
set -o pipefail
OUT=gpurun_out/r5q
mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-sensitivity"
for rep in 1 2; do
for cfg in "KDFM_X=0" "KDFM_WGR_CONV_WGS=128" "KDFM_WGR_CONV_WGS=64" "KDFM_WGRAD_CUS=224" "KDFM_WGRAD_CUS=192"; do
  env $cfg timeout -k 10 200 $B > $OUT/b.log 2>&1 || { echo "bench failed [$cfg]"; tail -5 $OUT/b.log; exit 3; }
  echo "[$cfg] $(tail -1 $OUT/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
