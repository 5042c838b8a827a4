# Parity of an A/B variant build (full-pass frames, graph/pipelined steps, the
# shipped chain) on DDQ_LIB_PATH=ab/$1, then the A/B timing of the variants
# named after it (tools/ab/run_ab.sh; "product" = the in-tree library)
set -e
mkdir -p gpurun_out
V=$1; shift
LIBP=$GRAFT_REPO_ROOT/distributed-deep-q_amd/ab/$V/libddq_hip.so
[ "$V" = product ] && LIBP=""
DDQ_LIB_PATH=$LIBP timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-full_pass or graph_step or pipelined or shipped or fused_apply}" > gpurun_out/var_parity_$V.log 2>&1 || { echo "PARITY_FAILED $V"; grep -E "FAILED|Error|assert" gpurun_out/var_parity_$V.log | head -20; tail -5 gpurun_out/var_parity_$V.log; exit 1; }
tail -1 gpurun_out/var_parity_$V.log
bash tools/ab/run_ab.sh "$@"
