#!/bin/bash
# round 5 final tree: GPU suite, smoke, the driver's bench line (20 steps) and a 30-step
# line, then the round's profiles (tools/gpu_r05p.sh: rocprofv3 stats + PMC passes)
set -o pipefail
D=gpurun_out/${1:-r05s}; mkdir -p $D
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit 2
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
timeout -k 10 300 python -u bench.py --gpus 1 --steps 30 --warmup 4 --no-legs --no-cpu-baseline > $D/bench_30.json 2> $D/bench_30.err || exit 4
tools/gpu_r05p.sh prof_${1:-r05s} || exit 5
