# Round 4, box 3: full GPU suite, a deepq16 (16x16 B=32) per-kernel line, then A/B variants
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
timeout -k 10 300 python bench.py --frame 16 --steps 2000 --warmup 100 --profile-steps 10 --chunks 10 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging > gpurun_out/bench_s16.json 2> gpurun_out/bench_s16.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_s16.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_s16.json
