#!/bin/bash
# round 5: node-path latency A/B (queues: latency-lane context, CU-masked queues, queue count)
set -o pipefail
D=gpurun_out/${1:-r05f}; mkdir -p $D
timeout -k 10 300 python -u tools/node_probe_r05.py $D/default 48 > $D/default.json 2> $D/default.err || exit 1
LB_PRIO_THREAD=0 timeout -k 10 300 python -u tools/node_probe_r05.py $D/nolane 48 > $D/nolane.json 2> $D/nolane.err || exit 2
LB_PRIO_CUS=0 timeout -k 10 300 python -u tools/node_probe_r05.py $D/nocus 48 > $D/nocus.json 2> $D/nocus.err || exit 3
LB_HW_QUEUES=12 timeout -k 10 300 python -u tools/node_probe_r05.py $D/q12 48 > $D/q12.json 2> $D/q12.err || exit 4
