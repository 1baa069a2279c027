#!/bin/bash
# round 5: GPU suite, then the driver's bench line, one-phase vs two-phase (combine) A/B
set -o pipefail
D=gpurun_out/${1:-r05d}; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 4 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 > $D/one_$k.json 2> $D/one_$k.err || exit 4
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 4 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 --combine on > $D/combine_$k.json 2> $D/combine_$k.err || exit 5
done
