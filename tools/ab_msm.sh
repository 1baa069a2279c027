#!/bin/bash
# A/B of the bucket MSM (default) against the per-set ladders (LB_MSM_MIN=0), alternating, 30 timed steps
set -e
mkdir -p gpurun_out/ab_msm
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 3 > gpurun_out/ab_msm/msm_$r.json 2> gpurun_out/ab_msm/msm_$r.err
  LB_MSM_MIN=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 3 > gpurun_out/ab_msm/ladder_$r.json 2> gpurun_out/ab_msm/ladder_$r.err
  echo "round $r ok"
done
