#!/bin/bash
# Run GPU steps in order, each under its own time limit; a test failure (exit 1) does not stop
# the sequence, anything else (a fault, an abort, a time limit) does.
# usage: tools/gpu_steps.sh OUTDIR 'cmd1' 'cmd2' ...   (each cmd's stdout/stderr -> OUTDIR/stepN.{out,err})
D=$1; shift; mkdir -p "$D"
i=0
for c in "$@"; do
  i=$((i + 1))
  bash -c "$c" > "$D/step$i.out" 2> "$D/step$i.err"
  rc=$?
  echo "step $i rc=$rc: $c" >> "$D/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after step $i (rc=$rc)" >> "$D/steps.txt"; exit $rc; fi
done
exit 0
