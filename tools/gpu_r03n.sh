#!/bin/bash
# r03n: lb_poll + the addon's non-blocking retire: poll test, JS-host GPU tests, node probe
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_js_host.py tests/test_gpu_same_message.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "poll or js or addon or node or same_message" > gpurun_out/r03n_tests.txt 2>&1
echo tests-ok
rm -rf gpurun_out/node_probe
timeout -k 10 600 python -u tools/node_probe.py gpurun_out/node_probe > gpurun_out/node_probe.log 2>&1
echo probe-ok
