#!/bin/bash
# Runtime knobs at 8 calls in flight: pairs per lane in k_miller_acc (LB_ACC_LPR 64 = 2 pairs, 32 = 4 pairs),
# k_lines waves/SIMD (LB_LINES_WAVES 1 | 2); 30 timed steps, two rounds
set -e
mkdir -p gpurun_out/ab_knobs8
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_knobs8/base_$r.json 2> /dev/null
  LB_ACC_LPR=32 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_knobs8/lpr32_$r.json 2> /dev/null
  LB_LINES_WAVES=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_knobs8/lw2_$r.json 2> /dev/null
  echo "round $r ok"
done
