#!/bin/bash
# End-of-round validation on the GPU box (what the driver runs): the whole GPU suite,
# smoke() and the driver's bench line.  usage (via gpurun): tools/gpu_validate.sh TAG
set -o pipefail
D=gpurun_out/${1:-validate}; mkdir -p $D
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $D/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 90 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_20.json 2> $D/bench_20.err || exit 3
echo done
