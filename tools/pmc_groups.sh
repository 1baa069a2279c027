#!/bin/bash
# PMC passes with caller-chosen counter groups over one C2 step (one call in
# flight); one rocprofv3 run per group (hardware limits per pass).
# usage: tools/pmc_groups.sh OUTDIR "GROUP1" "GROUP2" ...
set -e
OUT=$1; shift
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --steps 1 --warmup 0 --inflight 1 --sync"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pass$i -o pmc --output-format csv -- $CMD > $OUT.pass$i.log 2>&1
  echo "pass $i ($grp) ok"
done
