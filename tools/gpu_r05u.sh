#!/bin/bash
# round 5: why the 2-rank one-GPU rehearsal fell from 3.47 M (round 4) to 0.86 M --
# merged-check tail program off, two-phase release off, gt_check one-wave, fewer queues
set -o pipefail
D=gpurun_out/${1:-r05u}; mkdir -p $D
R="--gpus 2 --steps 10 --warmup 2 --no-legs --no-cpu-baseline --latency-reps 2 --iso-reps 0"
LB_MTAIL=0 timeout -k 10 300 python -u bench.py $R > $D/mtail0.json 2> $D/mtail0.err || exit 1
LB_TP_RELEASE=0 timeout -k 10 300 python -u bench.py $R > $D/tprel0.json 2> $D/tprel0.err || exit 2
LB_HW_QUEUES=8 timeout -k 10 300 python -u bench.py $R > $D/q8.json 2> $D/q8.err || exit 3
LB_MTAIL=0 LB_GT_LP=0 timeout -k 10 300 python -u bench.py $R > $D/mtail0_gt0.json 2> $D/mtail0_gt0.err || exit 4
