# GPU test subset ($PYTEST_K) then the A/B timing of the given variants
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab/run_ab.sh "$@"
