# GPU tests (optionally filtered by $PYTEST_K) + the default-length bench
# (no CPU leg / gather stress / sweep; with the world-1 exchange paths)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-stress --no-sweep > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json')); print('bench', d['value'], d['ms_per_step'], d['step_ms_distribution']); print(json.dumps(d['kernels_us']))
for k, v in d.get('exchange_paths', {}).get('paths', {}).items(): print(k, v['updates_per_s'], v['vs_exchange_free'], json.dumps(v.get('kernels_us')))"
