cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests.log 2>&1; echo tests_rc=$?
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; echo bench_rc=$?
cat gpurun_out/bench.json
