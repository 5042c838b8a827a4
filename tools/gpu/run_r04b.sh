# Round 4, box 2: exchange + host tests, the driver's bench invocation, the
# default line, a rocprofv3 kernel trace of the step chain alone, messaging.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_host.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_b.log | head -30; tail -5 gpurun_out/gpu_tests_b.log; exit 1; }
tail -1 gpurun_out/gpu_tests_b.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_driver.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_driver.json
timeout -k 10 400 python bench.py --no-cpu-baseline --no-gather-stress --no-sweep > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 3 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging > $R/gpurun_out/prof_step.json 2> $R/gpurun_out/prof_step.err
cd $R
python3 tools/trace_summary.py gpurun_out/prof_step step
