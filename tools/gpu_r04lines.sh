#!/bin/bash
# round-4: k_lines_rows at one or two waves per SIMD beside the LDS-accumulator step build
set -o pipefail
D=gpurun_out/${LB_OUT:-r04lines}; mkdir -p $D
B="python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3"
for r in 1 2 3; do
  timeout -k 10 300 $B > $D/default_$r.json 2> $D/default_$r.err || exit 1
  LB_LINES_WAVES=1 timeout -k 10 300 $B > $D/lines1_$r.json 2> $D/lines1_$r.err || exit 2
done
