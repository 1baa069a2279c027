#!/bin/bash
# round 5: the latency path at 64 rows per workgroup (1,024 threads, programs compiled for
# 64 rows: set 957 + final 379 rounds instead of 1,051 + 417) vs 32 rows
set -o pipefail
D=gpurun_out/${1:-r05y}; mkdir -p $D
V=$PWD/tools/variants_r05/lp64.so
LB_LIBRARY=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/lp64_tests.txt 2>&1 || exit 1
for k in 1 2; do
  LB_LP_BENCH_SIZES=1,128,1024 timeout -k 10 150 python -u tools/lp_bench.py 30 > $D/lp32_$k.txt 2>&1 || exit 2
  LB_LIBRARY=$V LB_LP_BENCH_SIZES=1,128,1024 timeout -k 10 150 python -u tools/lp_bench.py 30 > $D/lp64_$k.txt 2>&1 || exit 3
done
