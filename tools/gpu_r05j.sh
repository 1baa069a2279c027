#!/bin/bash
# round 5: node priority latency under load vs the node process's hardware-queue count
# (GPU_MAX_HW_QUEUES -> slots: 16 plain + 2 masked + 2 high-priority by default)
set -o pipefail
D=gpurun_out/${1:-r05j}; mkdir -p $D
for k in 1 2; do
  for q in 16 8; do
    GPU_MAX_HW_QUEUES=$q LB_NODE_FLAGS=" " timeout -k 10 300 python -u tools/node_probe_r05.py $D/q${q}_$k 48 > $D/q${q}_$k.json 2> $D/q${q}_$k.err || exit 1
  done
done
