#!/bin/bash
# r03m: steps parity tests (incl. a 1,200-set request in a merged call), the default bench
# line with the node leg after the bench's own context is closed (96 rounds)
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "steps or mixed or msm" > gpurun_out/r03m_tests.txt 2>&1
echo tests-ok
timeout -k 10 800 python -u bench.py > gpurun_out/r03m_bench_line.json 2> gpurun_out/r03m_bench.err
echo bench-ok
