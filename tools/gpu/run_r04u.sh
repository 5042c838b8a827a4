# Round 4, final code: the whole GPU suite, the driver's invocation, the
# default line, the full C3 sweep, the step kernel trace, the step-only PMC.
set -e
mkdir -p gpurun_out/u
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/u/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/u/gpu_tests.log | head -30; tail -5 gpurun_out/u/gpu_tests.log; exit 1; }
tail -1 gpurun_out/u/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/u/bench_driver.json 2> gpurun_out/u/bench_driver.err || { echo BENCH_FAILED; tail -20 gpurun_out/u/bench_driver.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/u/bench_driver.json > gpurun_out/u/bench_driver.txt
head -3 gpurun_out/u/bench_driver.txt
timeout -k 10 600 python bench.py > gpurun_out/u/bench.json 2> gpurun_out/u/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/u/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/u/bench.json > gpurun_out/u/bench.txt
cat gpurun_out/u/bench.txt
bash tools/gpu/run_r04_final.sh
