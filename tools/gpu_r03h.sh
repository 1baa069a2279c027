#!/bin/bash
# r03h: the steps organisation of the Miller accumulation (k_steps.hip): its parity tests,
# then an A/B against the pair-major k_miller_acc (LB_ACC=pairs), 30 timed steps each
set -e
mkdir -p gpurun_out/ab_r03h
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "steps or mixed or msm" > gpurun_out/r03h_tests.txt 2>&1
echo tests-ok
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 5 > gpurun_out/ab_r03h/steps_$r.json 2> gpurun_out/ab_r03h/steps_$r.err
  LB_ACC=pairs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 5 > gpurun_out/ab_r03h/pairs_$r.json 2> gpurun_out/ab_r03h/pairs_$r.err
  echo "round $r ok"
done
