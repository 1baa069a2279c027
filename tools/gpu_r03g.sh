#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03g_tests.txt 2>&1
echo tests-ok
bash tools/ab_r03g.sh
CMD="python3 bench.py --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --steps 1 --warmup 0 --inflight 1 --sync"
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -d gpurun_out/prof_r03g/lds -o pmc --output-format csv -- $CMD > gpurun_out/prof_r03g_lds.log 2>&1 && echo lds-pmc-ok
