#!/bin/bash
# round-4: latency-path round cost after grouping units by kind; priority-lane CU reservation A/B
set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 200 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_latency_path.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r04c/lp.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lp_probe.py > gpurun_out/r04c/lp_probe.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/lp_bench.py 30 > gpurun_out/r04c/lp_bench.log 2>&1 || exit 3
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/r04c/pmc -o lp -- python3 -u tools/lp_bench.py 5 > gpurun_out/r04c/pmc.log 2>&1 || exit 5
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c/trace -o lp -- python3 -u tools/lp_bench.py 30 > gpurun_out/r04c/trace.log 2>&1 || exit 6
for k in 0 8 16; do
  LB_PRIO_CUS=$k timeout -k 10 300 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --no-legs --iso-reps 0 > gpurun_out/r04c/bench_cus$k.json 2> gpurun_out/r04c/bench_cus$k.err || exit 4
done
