# detailed SQ counter passes over the eager bench (one pass per rocprofv3 run)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_WAVES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES" \
         "SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU"; do
  i=$((i+1))
  rm -rf $R/gpurun_out/pmc2_$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc2_$i -o p -- python3 $R/bench.py --steps 4 --warmup 2 --profile-steps 1 --no-cpu-baseline --no-gather-stress --eager > $R/gpurun_out/pmc2_$i.log 2>&1 || { echo PASS_$i FAILED; tail -5 $R/gpurun_out/pmc2_$i.log; exit 1; }
done
cd $R
python3 tools/pmc_detail.py gpurun_out/pmc2_1 gpurun_out/pmc2_2 gpurun_out/pmc2_3
