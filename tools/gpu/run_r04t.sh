# The next step's draw in the head launch: parity / chain / exchange / async
# suites, then the main line and 16x16 against the previous library (ab/base).
set -e
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_exchange.py tests/test_gpu_async.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/t/tests.log | head -30; tail -5 gpurun_out/t/tests.log; exit 1; }
tail -1 gpurun_out/t/tests.log
NOPARITY=1 STEPS=400 bash tools/gpu/run_ab.sh base
NOPARITY=1 FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh base
echo done
