# full-pass parity over the frame sweep, then per-kernel times at edge-tile
# and exact frames (tools/frame_kernels.py)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "full_pass" > gpurun_out/frames_parity.log 2>&1 || { echo PARITY_FAILED; tail -30 gpurun_out/frames_parity.log; exit 1; }
tail -3 gpurun_out/frames_parity.log
timeout -k 10 400 python3 -u tools/frame_kernels.py 256 32 40 64 72 104 > gpurun_out/fk256.jsonl 2> gpurun_out/fk.err
timeout -k 10 120 python3 -u tools/frame_kernels.py 32 16 64 > gpurun_out/fk32.jsonl 2>> gpurun_out/fk.err
cat gpurun_out/fk256.jsonl gpurun_out/fk32.jsonl
