# kernel trace of the default bench, then one PMC pass of the LDS counters
set -e
VARIANTS="0" bash tools/gpu/run_trace.sh
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_lds
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_lds -o p -- python3 $R/bench.py --steps 4 --warmup 2 --profile-steps 1 --no-cpu-baseline --no-gather-stress --eager > $R/gpurun_out/pmc_lds.log 2>&1 || { echo PMC_FAILED; tail -5 $R/gpurun_out/pmc_lds.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_lds/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "direct" in k or "wgrad" in k:
        bc = sum(d["SQ_LDS_BANK_CONFLICT"]) / max(1, len(d["SQ_LDS_BANK_CONFLICT"]))
        ia = sum(d["SQ_LDS_IDX_ACTIVE"]) / max(1, len(d["SQ_LDS_IDX_ACTIVE"]))
        print("%-70s conflict %.3g active %.3g (%.0f%%)" % (k, bc, ia, 100 * bc / max(ia, 1)))
PY
