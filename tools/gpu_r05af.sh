#!/bin/bash
# round 5: the lines kernel storing each doubling line before the point update -- parity
# suites, then two bench lines (iso stage times: k_lines_rows alone)
set -o pipefail
D=gpurun_out/${1:-r05af}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_multigpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/tests.txt 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --latency-reps 0 --iso-reps 3 > $D/b_$k.json 2> $D/b_$k.err || exit 2
done
