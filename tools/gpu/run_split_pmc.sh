# split-conv microbenchmark: timings of every config, then PMC passes of config $1
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 $R/tools/ubench/split_ubench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -i $R/tools/pmc_split.txt --output-format csv -d $R/gpurun_out/spmc -o spmc -- $R/tools/ubench/split_ubench ${1:-2} > /dev/null
cd $R
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob("gpurun_out/spmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "split_conv" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc):
    print("%-28s %14.4g per launch" % (k, acc[k] / max(1, n[k] / 1)))
PY
