#!/bin/bash
# round-4: the default bench line (legs included) with and without the priority-lane reservation
set -o pipefail
D=gpurun_out/${LB_OUT:-r04z}; mkdir -p $D
LB_PRIO_CUS=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline > $D/cus0.json 2> $D/cus0.err || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $D/default.json 2> $D/default.err || exit 2
