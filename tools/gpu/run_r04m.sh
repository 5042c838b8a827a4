# Round 4, final code: the whole GPU suite, the fc4-gradient debug print, then
# the final measurements (full C3 sweep, step kernel trace, step-only PMC).
set -e
mkdir -p gpurun_out/m
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/m/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/m/gpu_tests.log | head -30; tail -5 gpurun_out/m/gpu_tests.log; exit 1; }
tail -1 gpurun_out/m/gpu_tests.log
(cd distributed-deep-q_amd && timeout -k 10 200 python -u ../tools/gpu/dbg_grad64.py) > gpurun_out/m/dbg.log 2>&1 || { echo DBG_FAILED; tail -20 gpurun_out/m/dbg.log; exit 1; }
cat gpurun_out/m/dbg.log
bash tools/gpu/run_r04_final.sh
