#!/bin/bash
# round-4 GPU check: latency-path tests, parity, a short bench with the latency legs
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py tests/test_gpu_hwq.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04a/lp.log 2>&1 || exit 1
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a/parity.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-legs > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err || exit 3
timeout -k 10 200 python -u tools/lp_probe.py > gpurun_out/r04a/lp_probe.log 2>&1 || exit 4
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r04a/lp_prof -o lp -- python3 -u tools/lp_bench.py 30 > gpurun_out/r04a/lp_bench.log 2>&1 || exit 8
timeout -k 10 300 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --combine on > gpurun_out/r04a/bench_combine.json 2> gpurun_out/r04a/bench_combine.err || exit 5
timeout -k 10 300 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --combine off > gpurun_out/r04a/bench_onephase.json 2> gpurun_out/r04a/bench_onephase.err || exit 6
LB_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --gpus 2 --steps 16 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 > gpurun_out/r04a/bench_gpus2.json 2> gpurun_out/r04a/bench_gpus2.err || exit 7
