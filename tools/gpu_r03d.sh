#!/bin/bash
# full GPU suite (incl. the 1M-set 8-context C4 composition), full default bench, queue-count A/B
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_tests.txt 2>&1
echo tests-ok
timeout -k 10 600 python -u bench.py > gpurun_out/r03d_bench_line.json 2> gpurun_out/r03d_bench.err
echo bench-ok
bash tools/ab_hwq2.sh
