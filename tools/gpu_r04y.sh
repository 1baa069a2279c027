#!/bin/bash
# round-4: per-kernel iso timings of wave-count / step-mode variants
set -o pipefail
D=gpurun_out/${LB_OUT:-r04y}; mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 7
B="python -u bench.py --steps 24 --warmup 3 --no-cpu-baseline --no-legs --latency-reps 0 --iso-reps 3"
timeout -k 10 300 $B > $D/default.json 2> $D/default.err || exit 1
LB_LIBRARY=$PWD/tools/variants_r04/wh1/liblodestar_bls.so timeout -k 10 300 $B > $D/whash1.json 2> $D/whash1.err || exit 2
LB_LIBRARY=$PWD/tools/variants_r04/wm1/liblodestar_bls.so timeout -k 10 300 $B > $D/wmap1.json 2> $D/wmap1.err || exit 3
LB_STEP_MODE=0 LB_STEP_WAVES=1 timeout -k 10 300 $B > $D/step01.json 2> $D/step01.err || exit 4
LB_STEP_MODE=2 LB_STEP_WAVES=1 timeout -k 10 300 $B > $D/step21.json 2> $D/step21.err || exit 5
LB_STEP_MODE=1 LB_STEP_WAVES=1 timeout -k 10 300 $B > $D/step11.json 2> $D/step11.err || exit 6
timeout -k 10 600 python -u bench.py > $D/full.json 2> $D/full.err || exit 8
