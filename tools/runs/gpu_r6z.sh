set -o pipefail
OUT=gpurun_out/r6z
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; echo "smoke $?"; tail -3 $OUT/smoke.log
