#!/bin/bash
# round-5 GPU runs: the GPU suite, then the driver's bench command and a 30-step line.
# usage (on the box): tools/gpu_r05.sh OUTDIR [tests|bench|both]
set -o pipefail
D=gpurun_out/${1:-r05}; mkdir -p $D
MODE=${2:-both}
if [ "$MODE" != bench ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit 2
fi
if [ "$MODE" != tests ]; then
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 4 --no-legs --no-cpu-baseline > $D/bench_30.json 2> $D/bench_30.err || exit 4
fi
