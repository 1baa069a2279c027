#!/bin/bash
# default bench line (16 calls in flight, latency + node legs), op counts, gossip study, profiles
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r03e_bench_line.json 2> gpurun_out/r03e_bench.err
echo bench-ok
timeout -k 10 600 python -u tools/opcount.py --run --sets 16384 --out gpurun_out/op_counts_r03.json > gpurun_out/opcount.log 2>&1
echo opcount-ok
timeout -k 10 600 python -u tools/gossip_study.py > gpurun_out/gossip_study_r03.json 2> gpurun_out/gossip_study.err
echo gossip-ok
bash tools/prof_r03.sh r03e
