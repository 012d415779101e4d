#!/bin/bash
# HBM traffic of every kernel of the bench step from PMC counters (MI355X_MICROARCH.md §HBM):
# two separate rocprofv3 --pmc passes (FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2: they cannot share
# one pass), each with its own time limit; then tools/pmc_summary.py applies the gfx950 correction
# (FETCH_SIZE reports half the bytes of a 16-B/lane streaming read) and writes per-launch bytes.
# usage (repo root, via gpurun): bash tools/pmc_traffic.sh <tag>
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-sensitivity > "$OUT/fetch.log" 2>&1 &&
echo "fetch pass ok" &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-sensitivity > "$OUT/write.log" 2>&1 &&
echo "write pass ok" &&
python3 tools/pmc_summary.py "$OUT" > "$OUT/traffic.txt" && rm -rf "$OUT/fetch" "$OUT/write" && head -40 "$OUT/traffic.txt"
