#!/bin/bash
# round-4: k_step_acc organisation A/B, interleaved (default 2-wave one-line-at-a-time vs the
# one-wave LDS accumulator), then the PMC passes of the LDS-accumulator build
set -o pipefail
D=gpurun_out/${LB_OUT:-r04step}; mkdir -p $D
B="python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3"
for r in 1 2 3; do
  timeout -k 10 300 $B > $D/default_$r.json 2> $D/default_$r.err || exit 1
  LB_STEP_MODE=1 LB_STEP_WAVES=1 timeout -k 10 300 $B > $D/step11_$r.json 2> $D/step11_$r.err || exit 2
done
LB_STEP_MODE=1 LB_STEP_WAVES=1 bash tools/pmc.sh $D/pmc_step11 > $D/pmc.log 2>&1 || exit 3
python3 tools/pmc_summarize.py $D/pmc_step11 $D/pmc_traffic_step11.json > /dev/null || exit 4
