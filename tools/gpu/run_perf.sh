# parity (full pass + step) then the default bench without the slow extras
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in ${VARIANTS:-0}; do
DDQ_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-stress > gpurun_out/bench_v$v.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_v$v.json')); print('variant $v', d['value'], d['ms_per_step'], json.dumps(d['kernels_us']))"
done
