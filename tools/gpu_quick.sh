set -o pipefail
D=gpurun_out/r05i; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_block_sets.py tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread > $D/mem.txt 2>&1
echo "mem rc=$?"
LB_LIBRARY=tools/variants_r05/regs.so timeout -k 10 200 python -u -m pytest tests/test_gpu_block_sets.py -m gpu -v --timeout 120 --timeout-method thread > $D/regs.txt 2>&1
echo "regs rc=$?"
