#!/bin/bash
# round 5: node priority latency under load -- inputs generated in this process (its HIP
# queues opened and streams destroyed) vs in a child process (this one never opens one);
# the priority slot's buffers sized at lb_create
set -o pipefail
D=gpurun_out/${1:-r05k}; mkdir -p $D
for k in 1 2; do
  for c in 0 1; do
    LB_PROBE_CHILD_DATA=$c LB_NODE_FLAGS=" " timeout -k 10 300 python -u tools/node_probe_r05.py $D/c${c}_$k 48 > $D/c${c}_$k.json 2> $D/c${c}_$k.err || exit 1
  done
done
