set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/x32_parity.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error|assert" gpurun_out/x32_parity.log | head -20; tail -5 gpurun_out/x32_parity.log; exit 1; }
tail -2 gpurun_out/x32_parity.log
NOPARITY=1 STEPS=400 bash tools/gpu/run_ab.sh base
