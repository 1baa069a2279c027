set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_parity.py -k "msm or c2_full" -x -v --timeout 200 --timeout-method thread > gpurun_out/r03b_msm_tests.txt 2>&1
echo msm-tests-ok
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-legs > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err
echo bench-ok
