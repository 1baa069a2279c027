#!/bin/bash
# round 5: node onset/steady priority latency; 20-step line vs calls in flight
set -o pipefail
D=gpurun_out/${1:-r05g}; mkdir -p $D
timeout -k 10 300 python -u tools/node_probe_r05.py $D/node 48 > $D/node.json 2> $D/node.err || exit 1
for q in 8 12 16; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 --inflight $q > $D/b20_q$q.json 2> $D/b20_q$q.err || exit 2
done
