# Round 4: fc4 apply tiles with the x tile staged in LDS -- the step-chain
# suite (fused apply vs the oracle, bit-exact replays) on each variant, then
# the bench / rocprof A/B.  Usage: bash tools/gpu/run_r04y.sh v1 [v2 ...]
set -e
mkdir -p gpurun_out/ab
R=$GRAFT_REPO_ROOT
for V in "$@"; do
  DDQ_LIB_PATH=$R/distributed-deep-q_amd/ab/$V/libddq_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_exchange.py -x -q --timeout 300 --timeout-method thread -k "chain or no_grad_store or pipelined or graph or exchange or overlap or group" > gpurun_out/ab/chain_$V.log 2>&1 || { echo VARIANT_CHAIN_FAILED $V; tail -30 gpurun_out/ab/chain_$V.log; exit 1; }
  echo "[$V] $(tail -1 gpurun_out/ab/chain_$V.log)"
done
NOPARITY=1 bash tools/gpu/run_ab.sh "$@"
