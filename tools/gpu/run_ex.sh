set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
