#!/bin/bash
# round 5: two LP workgroups per CU by default; the round header in scalar registers vs
# vector (tools/variants_r05/lpvhdr.so) on the same box; the bench line (node onset)
set -o pipefail
D=gpurun_out/${1:-r05r}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/lp_tests.txt 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 120 python -u tools/lp_bench.py 40 > $D/lp_s_$k.txt 2>&1 || exit 2
  LB_LIBRARY=$PWD/tools/variants_r05/lpvhdr.so timeout -k 10 120 python -u tools/lp_bench.py 40 > $D/lp_v_$k.txt 2>&1 || exit 3
done
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_20.json 2> $D/bench_20.err || exit 4
