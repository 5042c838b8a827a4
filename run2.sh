cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/gpu_tests.log 2>&1; echo tests_rc=$?
tail -30 gpurun_out/gpu_tests.log
