# per-variant kernel durations from rocprofv3 kernel traces of the graph bench
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
fi
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-0}; do
  rm -rf $R/gpurun_out/tr_v$v
  DDQ_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_v$v -o run -- python3 $R/bench.py --steps 400 --warmup 20 --profile-steps 1 --no-cpu-baseline --no-gather-stress > $R/gpurun_out/tr_v$v.json 2> $R/gpurun_out/tr_v$v.err || { echo BENCH_FAILED; tail -20 $R/gpurun_out/tr_v$v.err; exit 1; }
  python3 $R/tools/trace_summary.py $R/gpurun_out/tr_v$v $v
done
