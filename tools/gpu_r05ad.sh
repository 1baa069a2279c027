#!/bin/bash
# round 5: k_step_acc builds in the final pipeline, interleaved, 3 rounds (20 steps, default flow)
set -o pipefail
D=gpurun_out/${1:-r05ad}; mkdir -p $D
B="--steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 3 --latency-reps 0"
for k in 1 2 3; do
  timeout -k 10 200 python -u bench.py $B > $D/default_$k.json 2> $D/default_$k.err || exit 1
  LB_STEP_MODE=2 LB_STEP_WAVES=2 timeout -k 10 200 python -u bench.py $B > $D/step2w2_$k.json 2> $D/step2w2_$k.err || exit 2
  LB_STEP_MODE=0 LB_STEP_WAVES=2 timeout -k 10 200 python -u bench.py $B > $D/step0w2_$k.json 2> $D/step0w2_$k.err || exit 3
done
