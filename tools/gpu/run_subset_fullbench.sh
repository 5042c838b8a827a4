# A test subset ($PYTEST_K) + the full default bench line (every section)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.json
