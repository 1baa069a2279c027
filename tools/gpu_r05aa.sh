#!/bin/bash
# round 5: JS host GPU tests (replays with PublicKey objects, e2e under load) and the bench
# line with the node leg (C4 PublicKey-object packing)
set -o pipefail
D=gpurun_out/${1:-r05aa}; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_js_host.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/js_tests.txt 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_20.json 2> $D/bench_20.err || exit 2
