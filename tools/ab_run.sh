#!/bin/bash
# A/B of tuning variants on the GPU box (one call, each step under its own limit).
# usage: tools/ab_run.sh TAG "NAME:ENV..." ...   (ENV may set LB_LIBRARY=..., LB_* knobs)
set -e
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
B="python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 --steps 30 --warmup 3 --iso-reps 1"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 $B > gpurun_out/${TAG}_${name}.json
done
