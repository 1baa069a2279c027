#!/bin/bash
# r03r: occupancy of the one-wave kernels: k_step_acc at 2 waves/SIMD (modes 0 and 2),
# k_lines_rows at 2 waves; steps parity under the 2-wave build, then the bench A/B
set -e
mkdir -p gpurun_out/ab_r03r
LB_STEP_WAVES=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "steps" > gpurun_out/r03r_tests.txt 2>&1
echo tests-ok
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03r/base_$r.json 2> /dev/null
  LB_STEP_WAVES=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03r/sw2_$r.json 2> /dev/null
  LB_STEP_WAVES=2 LB_STEP_MODE=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03r/sw2m2_$r.json 2> /dev/null
  LB_LINES_WAVES=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03r/lw2_$r.json 2> /dev/null
  echo "round $r ok"
done
