#!/bin/bash
# r03p: k_step_acc one line at a time (LB_STEP_MODE=2) vs paired lines (0): steps parity tests
# under mode 2, bench A/B (two rounds); then the node probe with the addon-side trace
set -e
mkdir -p gpurun_out/ab_r03p
LB_STEP_MODE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "steps or mixed or msm" > gpurun_out/r03p_tests.txt 2>&1
echo tests-ok
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03p/m0_$r.json 2> /dev/null
  LB_STEP_MODE=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 > gpurun_out/ab_r03p/m2_$r.json 2> /dev/null
  echo "round $r ok"
done
rm -rf gpurun_out/node_probe
timeout -k 10 600 python -u tools/node_probe.py gpurun_out/node_probe > gpurun_out/node_probe.log 2>&1
echo probe-ok
