#!/bin/bash
# round 5: k_hash_finish / k_decode_sigs at one wave per SIMD (no scratch: 402 VGPR+AGPR)
# against the 2-wave default; parity on the variant, then alternating bench lines
# (iso stage times name the kernels alone)
set -o pipefail
D=gpurun_out/${1:-r05ag}; mkdir -p $D
AB="--steps 20 --warmup 5 --no-legs --no-cpu-baseline --latency-reps 0 --iso-reps 3"
LB_LIBRARY=tools/variants_r05/hfdec1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/tests_hfdec1.txt 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 200 python -u bench.py $AB > $D/base_$k.json 2> $D/base_$k.err || exit 2
  for v in hf1 dec1 hfdec1; do
    LB_LIBRARY=tools/variants_r05/$v.so timeout -k 10 200 python -u bench.py $AB > $D/${v}_$k.json 2> $D/${v}_$k.err || exit 3
  done
done
echo done
