#!/bin/bash
# Round-3 first validation: GPU tests, smoke, default bench line.
set -e
TAG=${1:-r03a}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
echo "gpu tests ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench_line.json 2> gpurun_out/${TAG}_bench.err
echo "bench ok"
