#!/bin/bash
# round 5: node priority latency under load, per-call stage times of the 128-set priority jobs
set -o pipefail
D=gpurun_out/${1:-r05l}; mkdir -p $D
for k in 1 2; do
  LB_STAGE_EVENTS=1 LB_PROBE_CHILD_DATA=1 LB_NODE_FLAGS=" " timeout -k 10 300 python -u tools/node_probe_r05.py $D/s_$k 48 > $D/s_$k.json 2> $D/s_$k.err || exit 1
done
