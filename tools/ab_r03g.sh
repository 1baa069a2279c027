#!/bin/bash
# A/B on the LDS-padded build: calls in flight 16 / 24 / 32, and at 16: 4 pairs per lane in
# k_miller_acc (LB_ACC_LPR=32), 2-wave k_lines (LB_LINES_WAVES=2); 30 timed steps, two rounds
set -e
mkdir -p gpurun_out/ab_r03g
for r in 1 2; do
  for q in 16 24 32; do
    LB_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03g/q${q}_$r.json 2> gpurun_out/ab_r03g/q${q}_$r.err
  done
  LB_ACC_LPR=32 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03g/lpr32_$r.json 2> /dev/null
  LB_LINES_WAVES=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03g/lw2_$r.json 2> /dev/null
  echo "round $r ok"
done
