#!/bin/bash
# round-4: latency path after the single prefetch buffer (no global round trip per round)
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 200 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r04e/lp.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lp_probe.py > gpurun_out/r04e/lp_probe.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/lp_bench.py 30 > gpurun_out/r04e/lp_bench.log 2>&1 || exit 3
