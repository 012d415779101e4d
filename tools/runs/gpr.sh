#!/bin/bash
# run a gpurun call, waiting (up to ~12 min) while the pool reports no free box / slot (nothing ran, nothing charged)
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$rc" = 3 ] || [ "$st" = transient ]; then sleep 90; continue; fi
  exit $rc
done
exit $rc
