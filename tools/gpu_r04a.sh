#!/bin/bash
# round-4 GPU check: latency-path tests, parity, a short bench with the latency legs
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py tests/test_gpu_hwq.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04a/lp.log 2>&1 || exit 1
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a/parity.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-legs > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err || exit 3
timeout -k 10 200 python -u tools/lp_probe.py > gpurun_out/r04a/lp_probe.log 2>&1 || exit 4
