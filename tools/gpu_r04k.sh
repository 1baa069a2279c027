#!/bin/bash
# round-4: compact unit records (DPP broadcast) + priority-lane CU reservation spread over the CU ids
set -o pipefail
D=gpurun_out/${LB_OUT:-r04k}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_lp.py tests/test_gpu_latency_path.py tests/test_gpu_pubkey_table.py -x -q -s --timeout 120 --timeout-method thread > $D/lp.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lp_probe.py > $D/lp_probe.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/lp_bench.py 30 > $D/lp_bench.log 2>&1 || exit 3
for k in 16 32; do
  LB_PRIO_CUS=$k LB_PRIO_SPREAD=1 timeout -k 10 300 python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --no-legs --iso-reps 0 > $D/bench_spread$k.json 2> $D/bench_spread$k.err || exit 4
done
