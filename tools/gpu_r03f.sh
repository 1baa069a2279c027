#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03f_tests.txt 2>&1
echo tests-ok
timeout -k 10 600 python -u bench.py > gpurun_out/r03f_bench_line.json 2> gpurun_out/r03f_bench.err
echo bench-ok
timeout -k 10 600 python -u tools/gossip_study.py > gpurun_out/gossip_study_r03f.json 2> gpurun_out/gossip_study_f.err
echo gossip-ok
