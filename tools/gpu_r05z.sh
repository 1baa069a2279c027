#!/bin/bash
# round 5: a permanent 8-CU reservation for the priority lane (LB_PRIO_STATIC_CUS=8) vs none:
# C2 throughput, and the node leg's onset latency (first priority call after a quiet spell)
set -o pipefail
D=gpurun_out/${1:-r05z}; mkdir -p $D
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/default.json 2> $D/default.err || exit 1
LB_PRIO_STATIC_CUS=8 timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/static8.json 2> $D/static8.err || exit 2
