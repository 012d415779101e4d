# subsampling forward phase probe (built on the box: probe binaries are not pushed), depthwise micro
set -o pipefail
OUT=gpurun_out/r6k
mkdir -p $OUT
export PYTHONUNBUFFERED=1
hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/ss_probe.hip -L kd-via-fm-in-asr_amd/kdfm -lkdfm \
  -Wl,-rpath,'$ORIGIN/../kd-via-fm-in-asr_amd/kdfm' -o /tmp/ss_probe > $OUT/build.log 2>&1 || { echo build failed; exit 1; }
timeout -k 10 120 /tmp/ss_probe > $OUT/ss_probe.log 2>&1; echo "probe $?"
timeout -k 10 120 python tools/dwconv_micro.py > $OUT/dw_micro.log 2>&1; echo "dw $?"
