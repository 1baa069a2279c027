#!/bin/bash
# round 5: full bench line with the node leg run first (no HIP queue in the parent);
# 16 slots / 2 masked (default) vs 8 slots / 8 masked
set -o pipefail
D=gpurun_out/${1:-r05n}; mkdir -p $D
for g in 1 0; do LB_GT_LP=$g timeout -k 10 120 python -u tools/gt_probe.py > $D/gt_$g.json 2> $D/gt_$g.err || exit 3; done
for k in 1 2; do
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/q16_$k.json 2> $D/q16_$k.err || exit 1
  LB_HW_QUEUES=8 LB_PRIO_DYN_SLOTS=8 timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/q8_$k.json 2> $D/q8_$k.err || exit 2
done
