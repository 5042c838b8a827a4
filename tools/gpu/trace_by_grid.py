"""Per-grid-size durations of one kernel from a rocprofv3 kernel-trace CSV
(the launches of one kernel at several sizes, e.g. the replay gather at
n = 256 / 4096 / 32768): count, median and mean duration per grid.

usage: python tools/gpu/trace_by_grid.py <kernel_trace.csv> <name substring>"""
import csv
import statistics
import sys
from collections import defaultdict

path, name = sys.argv[1], sys.argv[2]
by = defaultdict(list)
for r in csv.DictReader(open(path)):
    if name not in r["Kernel_Name"]:
        continue
    g = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    by[g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for g in sorted(by):
    d = by[g]
    print("grid %s: %d launches, median %.2f us, mean %.2f us" % (g, len(d), statistics.median(d),
                                                                  statistics.mean(d)))
