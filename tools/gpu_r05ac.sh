#!/bin/bash
# round 5: runtime-knob sweep of the per-set organisation on the final tree (20 steps, the
# default two-phase flow): lines at 1 wave, step accumulation modes / waves
set -o pipefail
D=gpurun_out/${1:-r05ac}; mkdir -p $D
B="--steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0"
for k in 1 2; do
  timeout -k 10 200 python -u bench.py $B > $D/default_$k.json 2> $D/default_$k.err || exit 1
  LB_LINES_WAVES=1 timeout -k 10 200 python -u bench.py $B > $D/lines1_$k.json 2> $D/lines1_$k.err || exit 2
  LB_STEP_MODE=2 LB_STEP_WAVES=2 timeout -k 10 200 python -u bench.py $B > $D/step2w2_$k.json 2> $D/step2w2_$k.err || exit 3
  LB_STEP_MODE=0 timeout -k 10 200 python -u bench.py $B > $D/step0_$k.json 2> $D/step0_$k.err || exit 4
done
