#!/bin/bash
# round-4: two-phase calls with the host combine (resolver thread, gt_check off the lock) vs one-phase
set -o pipefail
D=gpurun_out/${LB_OUT:-r04x}; mkdir -p $D
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --combine on > $D/bench_combine.json 2> $D/bench_combine.err || exit 1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --combine off > $D/bench_onephase.json 2> $D/bench_onephase.err || exit 2
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --combine on > $D/bench_combine2.json 2> $D/bench_combine2.err || exit 3
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --combine off > $D/bench_onephase2.json 2> $D/bench_onephase2.err || exit 4
