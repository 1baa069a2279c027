#!/bin/bash
# Run a command on the MI355X box via gpurun; retry only when the box could not
# be prepared (status "transient": nothing ran, nothing charged).
# usage: [GPU_SH_TRIES=N] tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for attempt in $(seq 1 ${GPU_SH_TRIES:-4}); do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1 | tail -3
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ] && [ -n "$st" ]; then echo "[gpu.sh] status=$st"; exit 0; fi
  echo "[gpu.sh] transient, retrying in 45s"; sleep 45
done
exit 1
