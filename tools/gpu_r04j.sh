#!/bin/bash
# round-4: full GPU suite + small-call latency + throughput bench after the LP form/SHA changes
set -o pipefail
D=gpurun_out/${LB_OUT:-r04j}; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lp_probe.py > $D/lp_probe.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/lp_bench.py 30 > $D/lp_bench.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err || exit 4
