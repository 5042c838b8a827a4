# Round-end evidence in one call (product build): the full GPU suite, the
# default bench line (CPU leg, gather stress, C3 sweep), the acting bench, then
# tools/gpu/run_measure.sh (kernel-trace stats + one PMC pass per counter group).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_full.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --acting > gpurun_out/bench_acting.json 2> gpurun_out/bench_acting.err || { echo ACTING_FAILED; tail -20 gpurun_out/bench_acting.err; exit 1; }
bash tools/gpu/run_measure.sh > gpurun_out/measure.log 2>&1 || { echo MEASURE_FAILED; tail -20 gpurun_out/measure.log; exit 1; }
tail -3 gpurun_out/measure.log
