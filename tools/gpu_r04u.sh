#!/bin/bash
# round-4: the secondary legs with and without the priority-lane CU reservation
set -o pipefail
D=gpurun_out/${LB_OUT:-r04u}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_path.py tests/test_gpu_hwq.py tests/test_gpu_multigpu.py -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || exit 9
LB_PRIO_CUS=0 timeout -k 10 400 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --iso-reps 0 > $D/bench_cus0.json 2> $D/bench_cus0.err || exit 1
timeout -k 10 400 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --iso-reps 0 > $D/bench_default.json 2> $D/bench_default.err || exit 2
LB_PRIO_HOLD_MS=50 timeout -k 10 400 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --iso-reps 0 > $D/bench_hold50.json 2> $D/bench_hold50.err || exit 3
