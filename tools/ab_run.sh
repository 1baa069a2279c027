set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1_tests.txt 2>&1
B="python -u bench.py --no-cpu-baseline --no-legs --latency-reps 0 --steps 10 --warmup 2"
timeout -k 10 120 $B > gpurun_out/ab1_main.json
LB_LIBRARY=build/variants/scal_w1/liblodestar_bls.so timeout -k 10 120 $B > gpurun_out/ab1_w1.json
LB_LIBRARY=build/variants/scal_tab/liblodestar_bls.so timeout -k 10 120 $B > gpurun_out/ab1_tab.json
LB_LIBRARY=build/variants/scal_w1_tab/liblodestar_bls.so timeout -k 10 120 $B > gpurun_out/ab1_w1tab.json
timeout -k 10 120 $B > gpurun_out/ab1_main2.json
