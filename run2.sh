cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/gpu_tests.log 2>&1; echo tests_rc=$?
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; echo bench_rc=$?
cat gpurun_out/bench.json
DDQ_CONV_IMPL=gemm timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench_gemm.json 2> gpurun_out/bench.err; echo bench_rc=$?
cat gpurun_out/bench_gemm.json
