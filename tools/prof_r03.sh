#!/bin/bash
# Round-3 profiles on the GPU box: the integer-MAD peak microbenchmark, rocprofv3
# kernel stats of the bench with every call alone (--sync: the iso timing the
# roofline is priced on) and with calls in flight (the timed region), the PMC
# passes (tools/pmc.sh, incl. LDS bank conflicts of the MSM kernels) and a VALU
# instruction-mix pass; each step under its own limit.
set -e
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 120 tools/microbench/mad_rate > gpurun_out/prof_$TAG/mad_rate.txt 2>&1
echo "mad_rate ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/sync -o run --output-format csv -- \
  python3 bench.py --sync --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > gpurun_out/prof_$TAG/sync_line.json 2> gpurun_out/prof_$TAG/sync.err
echo "sync profile ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/pipe -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3 \
  > gpurun_out/prof_$TAG/pipe_line.json 2> gpurun_out/prof_$TAG/pipe.err
echo "pipelined profile ok"
tools/pmc.sh gpurun_out/prof_$TAG/pmc
echo "pmc ok"
# VALU instruction mix of every kernel (v_mad_u64_u32 share), and of the mad_rate
# microbenchmark as the calibration (its k_mad64 issues a known number of them)
CMD="python3 bench.py --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --steps 1 --warmup 0 --inflight 1 --sync"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES \
  -d gpurun_out/prof_$TAG/mix -o pmc --output-format csv -- $CMD > gpurun_out/prof_$TAG/mix.log 2>&1 \
  && echo "mix ok" || echo "mix pass failed (see mix.log)"
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES \
  -d gpurun_out/prof_$TAG/mix_cal -o pmc --output-format csv -- tools/microbench/mad_rate \
  > gpurun_out/prof_$TAG/mix_cal.log 2>&1 && echo "mix calibration ok" || echo "mix calibration failed"
