#!/bin/bash
# Round-end validation on the GPU box, each step under its own limit; stops at
# the first failure: all GPU tests, smoke(), the default bench line (with its
# cpu_baseline / C1 / host-API / adversarial / same-message legs), then the
# rocprofv3 kernel stats and PMC passes (tools/prof_r02.sh).
# usage: tools/final_r02.sh TAG
set -e
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
echo "gpu tests ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench_line.json 2> gpurun_out/${TAG}_bench.err
echo "bench ok"
bash tools/prof_r02.sh $TAG
