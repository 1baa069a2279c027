#!/bin/bash
# round 5: LP program stream from global memory by default -- GPU suite, smoke, the
# driver's bench line, then the round's profiles (tools/gpu_r05p.sh)
set -o pipefail
D=gpurun_out/${1:-r05q}; mkdir -p $D
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit 2
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
for k in 1 2; do
  LB_LP_BENCH_SIZES=1,128,512,1024 timeout -k 10 150 python -u tools/lp_bench.py 20 > $D/lp_v2_$k.txt 2>&1 || exit 4
  LB_LIBRARY=$PWD/tools/variants_r05/lpv4.so LB_LP_BENCH_SIZES=1,128,512,1024 timeout -k 10 150 python -u tools/lp_bench.py 20 > $D/lp_v4_$k.txt 2>&1 || exit 5
done
tools/gpu_r05p.sh prof_r05q || exit 6
