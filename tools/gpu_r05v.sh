#!/bin/bash
# round 5: 2-rank rehearsal with the per-rank queue split, and the N=1 combine A/B with a
# quarter more two-phase calls outstanding
set -o pipefail
D=gpurun_out/${1:-r05v}; mkdir -p $D
timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-legs --no-cpu-baseline --latency-reps 2 --iso-reps 0 > $D/gpus2.json 2> $D/gpus2.err || exit 1
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 > $D/one_$k.json 2> $D/one_$k.err || exit 2
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --iso-reps 0 --latency-reps 0 --combine on > $D/combine_$k.json 2> $D/combine_$k.err || exit 3
done
