# parity (direct full pass) + kernel trace for each DDQ_VARIANT in $VARIANTS
set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-0}; do
  DDQ_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "full_pass_parity and direct" --timeout 200 --timeout-method thread > gpurun_out/par_v$v.log 2>&1 || { echo PARITY_FAILED_v$v; grep -E "Error|assert" gpurun_out/par_v$v.log | head -10; exit 1; }
  echo "variant $v parity: $(tail -1 gpurun_out/par_v$v.log)"
done
SKIP_TESTS=1 bash tools/gpu/run_trace.sh
