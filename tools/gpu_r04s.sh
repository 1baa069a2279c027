#!/bin/bash
# round-4: priority lane with a CU reservation held only while the lane is in use (LB_PRIO_DYN);
# the masked streams take hardware queues of a pool of their own (scratch per queue, §5.1):
# 16 unmasked queues + K masked streams (LB_PRIO_DYN_SLOTS)
set -o pipefail
D=gpurun_out/${LB_OUT:-r04s}; mkdir -p $D
CFGS=${LB_CFGS:-"16_16_1_4 16_16_1_6 16_0_0_0"}
for c in $CFGS; do
  cfg=${c//_/ }
  set -- $cfg
  LB_HW_QUEUES=$1 LB_PRIO_CUS=$2 LB_PRIO_DYN=$3 LB_PRIO_DYN_SLOTS=$4 timeout -k 10 300 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --no-legs --iso-reps 0 > $D/bench_q$1_cus$2_dyn$3_s$4.json 2> $D/bench_q$1_cus$2_dyn$3_s$4.err || exit 2
done
