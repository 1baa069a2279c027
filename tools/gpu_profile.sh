#!/bin/bash
# Profiles of the bench: rocprofv3 kernel stats with every call alone (--sync,
# LB_DAG=0: the iso timings the roofline is priced on) and of the pipelined timed region, then
# the HBM-traffic PMC passes of one C2 call (tools/pmc.sh; summarise with tools/pmc_summarize.py).
# usage (via gpurun): tools/gpu_profile.sh TAG
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-prof}; mkdir -p $D
LB_DAG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/sync -o run --output-format csv -- \
  python3 bench.py --sync --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > $D/sync_line.json 2> $D/sync.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/pipe -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > $D/pipe_line.json 2> $D/pipe.err || exit 2
tools/pmc.sh $D/pmc > $D/pmc.log 2>&1 || exit 3
echo done
