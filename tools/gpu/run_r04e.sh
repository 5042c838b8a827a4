set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_e.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests_e.log; exit 1; }
tail -1 gpurun_out/gpu_tests_e.log
FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh nofork
mkdir -p gpurun_out/ab64 
FRAME=64 STEPS=400 bash tools/gpu/run_ab.sh nofork
echo done
