#!/bin/bash
# Run several GPU steps in one gpurun call; each step gets its own time limit.
# A step that ends with a test failure (rc 1) lets the next step run; a timeout,
# abort, segfault or any other status ends the call there.
# usage: tools/gpu_steps.sh SECONDS 'cmd1' 'cmd2' ...
T=$1; shift
i=0
for c in "$@"; do
  i=$((i+1))
  echo "[step $i] $c"
  timeout -k 10 "$T" bash -c "$c"
  rc=$?
  echo "[step $i] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_steps] stopping after rc=$rc"; exit $rc; fi
done
