# Round 4, last code: smoke, the whole GPU suite, the driver's invocation and
# the default line.
set -e
mkdir -p gpurun_out/x
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/x/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/x/smoke.log; exit 1; }
tail -1 gpurun_out/x/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/x/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/x/gpu_tests.log; exit 1; }
tail -1 gpurun_out/x/gpu_tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/x/bench_driver.json 2> gpurun_out/x/bench_driver.err
python3 tools/bench_summary.py gpurun_out/x/bench_driver.json | head -3
timeout -k 10 600 python bench.py > gpurun_out/x/bench.json 2> gpurun_out/x/bench.err
python3 tools/bench_summary.py gpurun_out/x/bench.json | head -3
echo done
