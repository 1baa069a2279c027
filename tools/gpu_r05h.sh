#!/bin/bash
# round 5: register-spill cuts (memory-parked points in hash_finish, decode_sigs,
# lines) -- GPU suite, bench line, A/B against the register-resident variant
# (tools/variants_r05/regs.so: -DLB_HASH_FINISH_REGS -DLB_DECODE_REGS -DLB_LINES_QREGS),
# HBM traffic of both, kernel-trace stats of the default build.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r05h}; mkdir -p $D
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
AB="--steps 30 --warmup 4 --no-legs --no-cpu-baseline --latency-reps 0 --iso-reps 3"
for k in 1 2; do
  timeout -k 10 200 python -u bench.py $AB > $D/mem_$k.json 2> $D/mem_$k.err || exit 4
  LB_LIBRARY=tools/variants_r05/regs.so timeout -k 10 200 python -u bench.py $AB > $D/regs_$k.json 2> $D/regs_$k.err || exit 5
done
tools/pmc_traffic_ab.sh $D/pmc "mem:-" "regs:$PWD/tools/variants_r05/regs.so" > $D/pmc.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_sync -o run --output-format csv -- \
  python3 bench.py --sync --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > $D/prof_sync_line.json 2> $D/prof_sync.err || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_pipe -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > $D/prof_pipe_line.json 2> $D/prof_pipe.err || exit 8
echo done
