#!/bin/bash
# round-4: latency path with the branch-on-ripple normalisation
set -o pipefail
D=gpurun_out/${LB_OUT:-r04g}; mkdir -p $D
timeout -k 10 200 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_lp.py tests/test_gpu_latency_path.py -x -q -s --timeout 120 --timeout-method thread > $D/lp.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lp_probe.py > $D/lp_probe.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/lp_bench.py 30 > $D/lp_bench.log 2>&1 || exit 3
