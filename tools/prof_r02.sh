#!/bin/bash
# Round-2 profiles on the GPU box: rocprofv3 kernel stats of the bench with every
# call alone (--sync: the iso timing the roofline is priced on) and with 4 calls
# in flight (the headline's timed region), then the PMC passes (tools/pmc.sh).
set -e
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/sync -o run --output-format csv -- \
  python3 bench.py --sync --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > gpurun_out/prof_$TAG/sync_line.json 2> gpurun_out/prof_$TAG/sync.err
echo "sync profile ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/pipe -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > gpurun_out/prof_$TAG/pipe_line.json 2> gpurun_out/prof_$TAG/pipe.err
echo "pipelined profile ok"
tools/pmc.sh gpurun_out/prof_$TAG/pmc
echo "pmc ok"
