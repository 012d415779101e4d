# rehearsal of the driver's N>1 bench launch on one GPU: 2 ranks over gloo (KDFM_DIST_BACKEND=gloo), same script
set -o pipefail
OUT=gpurun_out/r6af
mkdir -p $OUT
export PYTHONUNBUFFERED=1 KDFM_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-f32-sensitivity > $OUT/bench2.log 2>&1; echo "rc $?"
tail -1 $OUT/bench2.log | cut -c1-400
