# parity tests, then kernel traces of the graph bench and the pipelined bench
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
for m in graph pipe; do
  x="--no-pipeline"; [ $m = pipe ] && x=""
  rm -rf $R/gpurun_out/tr_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_$m -o run -- python3 $R/bench.py --steps 400 --warmup 20 --profile-steps 1 --no-cpu-baseline --no-gather-stress $x > $R/gpurun_out/tr_$m.json 2> $R/gpurun_out/tr_$m.err || { echo BENCH_FAILED; tail -20 $R/gpurun_out/tr_$m.err; exit 1; }
  python3 $R/tools/trace_summary.py $R/gpurun_out/tr_$m $m
done
timeout -k 10 300 python3 $R/bench.py --no-gather-stress --no-cpu-baseline > $R/gpurun_out/bench_pipe.json 2> $R/gpurun_out/bench_pipe.err && python3 -c "import json; d=json.load(open('$R/gpurun_out/bench_pipe.json')); print('pipe bench', d['value'], d['ms_per_step'], d.get('step_ms_distribution'))"
