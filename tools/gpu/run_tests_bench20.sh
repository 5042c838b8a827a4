# GPU tests + the driver's short bench shape (20 steps, 5 warm-up)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gather-stress --chunks 0 --profile-steps 2 > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench20.json')); print('bench20', d['value'], d['ms_per_step'])"
