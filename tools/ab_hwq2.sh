#!/bin/bash
# A/B of the hardware-queue count (library slots = calls in flight): 8 / 12 / 16, 30 timed steps
set -e
mkdir -p gpurun_out/ab_hwq2
for r in 1 2; do
  for q in 8 12 16; do
    LB_HW_QUEUES=$q LB_SLOTS=$q timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 3 --inflight $q > gpurun_out/ab_hwq2/q${q}_$r.json 2> gpurun_out/ab_hwq2/q${q}_$r.err
  done
  echo "round $r ok"
done
