#!/bin/bash
# Run a command on the MI355X box via gpurun; retry only when the box could not be
# prepared (status "transient": nothing ran, nothing charged), up to 10 times.
# usage: tools/gpu_retry.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1 | grep -v "every call sends" | tail -3
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ] && [ -n "$st" ]; then echo "[gpu_retry] status=$st"; exit 0; fi
  echo "[gpu_retry] transient (attempt $attempt), retrying in 90s"; sleep 90
done
exit 1
