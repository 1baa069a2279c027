#!/bin/bash
# A/B: 4 hardware queues (HIP default, 4 slots) vs GPU_MAX_HW_QUEUES=8 (8 slots), 30 timed steps
set -e
mkdir -p gpurun_out/ab_hwq
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 3 > gpurun_out/ab_hwq/q4_$r.json 2> gpurun_out/ab_hwq/q4_$r.err
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 3 > gpurun_out/ab_hwq/q8_$r.json 2> gpurun_out/ab_hwq/q8_$r.err
  echo "round $r ok"
done
