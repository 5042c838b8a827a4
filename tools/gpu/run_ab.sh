# A/B of tuning variants (experiment build): parity of the full pass under
# each of $PARITY_VARIANTS, then kernel traces of the graph bench for each of $ENVS.
set -e
mkdir -p gpurun_out
for v in ${PARITY_VARIANTS:-0}; do
  DDQ_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "${PYTEST_K:-full_pass}" > gpurun_out/ab_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; grep -E "FAILED|Error|assert" gpurun_out/ab_tests_$v.log | head -30; tail -5 gpurun_out/ab_tests_$v.log; exit 1; }
  echo "parity variant $v: $(tail -1 gpurun_out/ab_tests_$v.log)"
done
bash tools/gpu/run_knobs.sh
