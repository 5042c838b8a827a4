set -e
mkdir -p gpurun_out
DDQ_VARIANT=${TEST_VARIANT:-0} timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in ${VARIANTS:-0}; do
  DDQ_VARIANT=$v timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err
  python - $v <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/bench_v{sys.argv[1]}.json"))
print("variant",sys.argv[1],d["value"],d["ms_per_step"],json.dumps(d["kernels_us"]))
PY
done
