#!/bin/bash
# full GPU test suite on the current build, then the hardware-queue A/B
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03c_tests.txt 2>&1
echo tests-ok
bash tools/ab_hwq.sh
