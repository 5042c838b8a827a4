set -e
for i in 1 2; do
timeout -k 10 200 python tools/gpu/ticket_prof.py 64 400 > gpurun_out/tp_prod_$i.log 2>&1
DDQ_LIB_PATH=$GRAFT_REPO_ROOT/distributed-deep-q_amd/ab/base/libddq_hip.so timeout -k 10 200 python tools/gpu/ticket_prof.py 64 400 > gpurun_out/tp_base_$i.log 2>&1
done
tail -2 gpurun_out/tp_*.log
