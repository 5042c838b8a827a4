# full-pass parity over the frame sweep, then the A/B timing of the given
# variants (tools/ab/run_ab.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "full_pass or fused_apply or graph_step or pipelined" > gpurun_out/parity_ab.log 2>&1 || { echo PARITY_FAILED; tail -30 gpurun_out/parity_ab.log; exit 1; }
tail -1 gpurun_out/parity_ab.log
bash tools/ab/run_ab.sh "$@"
