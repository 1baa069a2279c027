#!/bin/bash
# round 5: the bench line with the two-phase flow by default (20 steps with every leg, 30
# steps main line), and one rocprofv3 stats pass of the pipelined timed region
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r05w}; mkdir -p $D
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 30 --warmup 4 --no-legs --no-cpu-baseline > $D/bench_30.json 2> $D/bench_30.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/pipe -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 \
  > $D/pipe_line.json 2> $D/pipe.err || exit 3
