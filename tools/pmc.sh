#!/bin/bash
# PMC passes over one C2 step (65,536 sets, one call in flight so launches do
# not overlap); one counter group per rocprofv3 run (the hardware limits per
# pass: <= 8 SQ, <= 4 TCC counters; FETCH_SIZE uses 3 TCC, WRITE_SIZE 2).
# Runs on the GPU box:  tools/pmc.sh OUTDIR   then   python tools/pmc_summarize.py OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$(dirname "$OUT")" "$OUT"
export TMPDIR=/tmp
export LB_DAG=0  # one stream: the kernels of a call one after the other
CMD="python3 bench.py --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --steps 1 --warmup 0 --inflight 1 --sync"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pass$i -o pmc --output-format csv -- $CMD > $OUT.pass$i.log 2>&1
  echo "pass $i ($grp) ok"
done
