# Round 4, final-code box 1: the whole GPU suite, then the bench's default
# line (every leg: deepq16, C3 frames, exchange paths, messaging, gather
# stress, CPU baseline) and the driver's own invocation.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_h.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_h.log | head -30; tail -5 gpurun_out/gpu_tests_h.log; exit 1; }
tail -1 gpurun_out/gpu_tests_h.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_h.json 2> gpurun_out/bench_driver_h.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_driver_h.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_driver_h.json
timeout -k 10 600 python bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_h.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_h.json
echo done
