#!/bin/bash
# round 5: (1) lb_gt_check alone, round program vs one wave; (2) the latency path with the
# program stream read straight from global memory (LB_LP_DIRECT, tools/variants_r05/lpdirect.so)
# vs the LDS ring: its GPU tests and lone-call p50s; (3) the full bench line with the node leg
# run first, 16 slots / 2 masked (default) vs 8 slots / 8 masked
set -o pipefail
D=gpurun_out/${1:-r05n}; mkdir -p $D
V=$PWD/tools/variants_r05/lpdirect.so
for g in 1 0; do LB_GT_LP=$g timeout -k 10 120 python -u tools/gt_probe.py > $D/gt_$g.json 2> $D/gt_$g.err || exit 1; done
LB_LIBRARY=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/lpdirect_tests.txt 2>&1 || exit 2
for k in 1 2; do
  timeout -k 10 120 python -u tools/lp_bench.py 40 > $D/lp_ring_$k.txt 2>&1 || exit 3
  LB_LIBRARY=$V timeout -k 10 120 python -u tools/lp_bench.py 40 > $D/lp_direct_$k.txt 2>&1 || exit 4
done
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/q16_1.json 2> $D/q16_1.err || exit 5
LB_HW_QUEUES=8 LB_PRIO_DYN_SLOTS=8 timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/q8_1.json 2> $D/q8_1.err || exit 6
