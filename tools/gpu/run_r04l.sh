# Debug of the fc4 gradient block at S=64, then the parity / chain / host
# suites (branchless w1 routing loads, C1 value checks, no-grad-store flag),
# then A/Bs: conv1 tiles, fused conv1 wgrad cost (timing only), zero-filled
# dconv1 image, small-map conv2 forward with two k groups.
set -e
mkdir -p gpurun_out/l
(cd distributed-deep-q_amd && timeout -k 10 200 python -u ../tools/gpu/dbg_grad64.py) > gpurun_out/l/dbg.log 2>&1 || { echo DBG_FAILED; tail -20 gpurun_out/l/dbg.log; exit 1; }
cat gpurun_out/l/dbg.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_host.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/l/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/l/tests.log | head -30; tail -5 gpurun_out/l/tests.log; exit 1; }
tail -1 gpurun_out/l/tests.log
STEPS=400 bash tools/gpu/run_ab.sh c1t16 c1t20 c1t24 w1zf
NOPARITY=1 STEPS=400 bash tools/gpu/run_ab.sh now1
FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh c2fwk2
echo done
