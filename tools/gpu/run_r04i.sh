# fc4 data gradient as n-quarter partials: parity / chain / exchange suites on
# the product, then the A/B against the previous library (ab/base) at 64x64
# and 16x16.
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_exchange.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_i.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_i.log | head -30; tail -5 gpurun_out/gpu_tests_i.log; exit 1; }
tail -1 gpurun_out/gpu_tests_i.log
NOPARITY=1 STEPS=400 bash tools/gpu/run_ab.sh base
NOPARITY=1 FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh base
echo done
