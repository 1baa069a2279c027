#!/bin/bash
# r03j: k_step_acc with its accumulator in registers (default) vs in LDS (LB_STEP_LDS=1):
# the steps parity tests under both, then an A/B of the bench (30 timed steps, iso timings
# on a single-stream context), two rounds
set -e
mkdir -p gpurun_out/ab_r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "steps or mixed or msm" > gpurun_out/r03j_tests.txt 2>&1
LB_STEP_LDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "steps or mixed or msm" > gpurun_out/r03j_tests_lds.txt 2>&1
echo tests-ok
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03j/reg_$r.json 2> gpurun_out/ab_r03j/reg_$r.err
  LB_STEP_LDS=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03j/lds_$r.json 2> gpurun_out/ab_r03j/lds_$r.err
  echo "round $r ok"
done
