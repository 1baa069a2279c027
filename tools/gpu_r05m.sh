#!/bin/bash
# round 5: priority-slot copies as kernels -- GPU suite, node probe x2, full bench line
set -o pipefail
D=gpurun_out/${1:-r05m}; mkdir -p $D
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
for k in 1 2; do
  LB_STAGE_EVENTS=1 LB_PROBE_CHILD_DATA=1 LB_NODE_FLAGS=" " timeout -k 10 300 python -u tools/node_probe_r05.py $D/s_$k 48 > $D/s_$k.json 2> $D/s_$k.err || exit 2
done
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
