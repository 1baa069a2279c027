#!/bin/bash
# Round-3 final evidence: the full GPU suite, smoke(), the default bench line, a
# single-stream rocprofv3 kernel-stats profile of the same bench (the roofline's timing)
set -e
export TMPDIR=/tmp
TAG=${TAG:-r03z}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
echo smoke-ok
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench_line.json 2> gpurun_out/${TAG}_bench.err
echo bench-ok
LB_DAG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/sync -o run --output-format csv -- \
  python3 bench.py --sync --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > gpurun_out/prof_$TAG/sync_line.json 2> gpurun_out/prof_$TAG/sync.err
echo prof-ok
