export PROF="--steps 400 --warmup 20 --no-cpu-baseline --no-gather-stress --no-sweep --no-messaging --no-exchange-paths --chunks 0 --profile-steps 5 --no-isolated --preheat-ms 0"
export PMC="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY;SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
bash tools/gpu/run.sh
