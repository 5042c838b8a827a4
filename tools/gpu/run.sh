# One parameterised GPU-box runner (replaces the one-off run_r04*.sh scripts).
# Every step is bounded by its own timeout and the chain stops at the first
# failure (no GPU step after a fault / abort / time limit).
#   TESTS="expr"   pytest -m gpu -k expr over tests/ ("all": the whole GPU suite)
#   TFILES="..."   restrict the test files (default tests/)
#   BENCH="args"   python bench.py args -> gpurun_out/bench.json (+ .err)
#   PROF="args"    rocprofv3 --kernel-trace --stats of bench.py args -> gpurun_out/prof
#   PMC="ctrs"     one rocprofv3 --pmc pass per ';'-separated counter set over
#                  bench.py $PROF args -> gpurun_out/pmc_<i>
set -e
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$PWD}
if [ -n "$TESTS" ]; then
  K=""; [ "$TESTS" != all ] && K="$TESTS"
  timeout -k 10 ${TTIME:-900} python -u -m pytest ${TFILES:-tests/} -x -v -s -m gpu --timeout 300 \
    --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1 || {
    echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30
    tail -5 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BTIME:-300} python bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err || {
    echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
  python tools/bench_summary.py gpurun_out/bench.json | head -20
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run \
    -- python3 $R/bench.py $PROF > $R/gpurun_out/prof.json 2> $R/gpurun_out/prof.err || {
    echo PROF_FAILED; tail -5 $R/gpurun_out/prof.err; exit 1; }
  cd $R
  python3 tools/trace_summary.py gpurun_out/prof prof | head -40
  # (the per-dispatch trace stays on the box: gpurun_out is merged back <= 64 MiB)
  find gpurun_out/prof -name "*kernel_trace.csv" -size +8M -delete
fi
if [ -n "$PMC" ]; then
  i=0
  IFS=';' read -ra SETS <<< "$PMC"
  for C in "${SETS[@]}"; do
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_$i -o run \
      -- python3 $R/bench.py $PROF > /dev/null 2> $R/gpurun_out/pmc_$i.err || {
      echo PMC_FAILED $i; tail -5 $R/gpurun_out/pmc_$i.err; exit 1; }
    cd $R
    i=$((i + 1))
  done
  # per-kernel means of every pass -> one JSON (tools/pmc_json.py), raw rows dropped
  python3 tools/pmc_json.py gpurun_out gpurun_out/pmc.json
  find gpurun_out -path "*pmc_*" -name "*.csv" -delete
fi
