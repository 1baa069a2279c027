#!/bin/bash
# ${TAG}: full GPU suite, op counts of the steps organisation, single-stream rocprof kernel
# stats (the iso timings the roofline is priced on), the default bench line, PMC passes
set -e
TAG=${TAG:-r03k}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_${TAG}
[ -n "$TESTS" ] && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
echo tests-ok
[ -n "$OPCOUNT" ] && timeout -k 10 300 python -u tools/opcount.py --run --sets 16384 --out gpurun_out/op_counts_${TAG}.json > gpurun_out/opcount_${TAG}.log 2>&1
[ -n "$OPCOUNT" ] && cp gpurun_out/op_counts_${TAG}.json profiles/op_counts.json
echo opcount-ok
LB_DAG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}/sync -o run --output-format csv -- \
  python3 bench.py --sync --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > gpurun_out/prof_${TAG}/sync_line.json 2> gpurun_out/prof_${TAG}/sync.err
echo sync-prof-ok
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench_line.json 2> gpurun_out/${TAG}_bench.err
echo bench-ok
[ -n "$PMC" ] && tools/pmc.sh gpurun_out/prof_${TAG}/pmc
[ -n "$PMC" ] && python3 tools/pmc_summarize.py gpurun_out/prof_${TAG}/pmc gpurun_out/prof_${TAG}/pmc_traffic_${TAG}.json > /dev/null
echo pmc-ok
