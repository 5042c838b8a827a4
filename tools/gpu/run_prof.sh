set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --profile-steps 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print("%-60s %6s %10.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1000))
PY
