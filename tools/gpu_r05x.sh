#!/bin/bash
# round 5: one-phase calls with the merged-check program on the high-priority aux stream
# (LB_TAIL_AUX=1) vs on the call's own stream; parity with it on
set -o pipefail
D=gpurun_out/${1:-r05x}; mkdir -p $D
LB_TAIL_AUX=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/tests_aux.txt 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 --combine off > $D/one_$k.json 2> $D/one_$k.err || exit 2
  LB_TAIL_AUX=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 --combine off > $D/aux_$k.json 2> $D/aux_$k.err || exit 3
done
