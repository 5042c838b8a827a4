"""Per-kernel PMC averages (per dispatch) from a rocprofv3 counter-collection
directory: python3 tools/pmc_kernels.py DIR [name-substring]."""
import collections
import csv
import glob
import sys

root, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if filt and filt not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k[:110])
    for c in sorted(cs):
        v = cs[c]
        print("   %-28s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
