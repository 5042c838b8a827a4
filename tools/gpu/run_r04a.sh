# Round 4, first box: full GPU suite, the driver's bench invocation, the
# 500-step default line (no CPU / gather / sweep legs), and a rocprofv3
# kernel trace of the step chain alone.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_driver.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-gather-stress --no-sweep > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths > $R/gpurun_out/prof_step.json 2> $R/gpurun_out/prof_step.err
cd $R
python3 tools/trace_summary.py gpurun_out/prof_step step
python3 tools/bench_summary.py gpurun_out/bench_driver.json
python3 tools/bench_summary.py gpurun_out/bench.json
timeout -k 10 240 python -c "import json, bench; print(json.dumps(bench.messaging_costs()))" > gpurun_out/messaging.json 2> gpurun_out/messaging.err || { echo MESSAGING_FAILED; tail -20 gpurun_out/messaging.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/messaging.json'))
for f in d['frames']: print(f['frame'], f['raw'], f['server'])"
