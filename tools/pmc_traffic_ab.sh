#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE) over one C2 call for several
# library variants, to set per-stage spill traffic beside stage times.
# usage: tools/pmc_traffic_ab.sh OUTDIR "NAME:LIBRARY_PATH_OR_-" ...
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 0 --steps 1 --warmup 0 --inflight 1 --sync"
for spec in "$@"; do
  name=${spec%%:*}; lib=${spec#*:}
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    if [ "$lib" = "-" ]; then
      timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/$name/pass$i -o pmc --output-format csv -- $CMD > $OUT/$name.pass$i.log 2>&1
    else
      LB_LIBRARY=$lib timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/$name/pass$i -o pmc --output-format csv -- $CMD > $OUT/$name.pass$i.log 2>&1
    fi
    echo "$name pass $i ($grp) ok"
  done
done
