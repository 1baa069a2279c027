#!/bin/bash
# r03s: both occupancy changes together (k_lines_rows and k_step_acc one-line at 2 waves/SIMD)
# against the default, three rounds each
set -e
mkdir -p gpurun_out/ab_r03s
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03s/base_$r.json 2> /dev/null
  LB_LINES_WAVES=2 LB_STEP_WAVES=2 LB_STEP_MODE=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03s/both_$r.json 2> /dev/null
  echo "round $r ok"
done
