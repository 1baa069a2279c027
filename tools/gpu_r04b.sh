#!/bin/bash
# round-4 node-path probe: prefetch depths, loaded latency legs, the JS host's CPU ceiling
set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 120 node tools/js_host_bench.js 8 16 > gpurun_out/r04b/js_host_bench.json 2>&1 || exit 1
LB_PROBE_PREFETCH=0,1,2 LB_PROBE_ROUNDS=48 timeout -k 10 900 python -u tools/node_probe.py gpurun_out/r04b/node > gpurun_out/r04b/node_probe.log 2>&1 || exit 2
