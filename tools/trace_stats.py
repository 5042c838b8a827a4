"""Per-kernel duration statistics of ONE segment of a rocprofv3 kernel trace,
in the layout of rocprofv3's own kernel_stats.csv.

bench.py's profiled run dispatches every step kernel first inside the graph
replays (warmup + timed steps), then --profile-steps eager steps whose
kernels carry hipExtLaunchKernel start/stop events (the line's per-kernel
in-step times).  rocprofv3's --stats averages both together; this splits
them: the LAST <n> dispatches of each kernel are the eager profile steps.

Usage: python tools/trace_stats.py <trace.csv> <n_eager> eager|graph > out.csv"""
import collections
import csv
import statistics
import sys


def main():
    path, n, seg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]),
                                      int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for name, v in per.items():
        v.sort()
        if len(v) <= n:
            continue                      # not a step kernel (setup copies, fills)
        d = [x for _, x in (v[-n:] if seg == "eager" else v[:-n])]
        rows.append((name, len(d), sum(d), sum(d) / len(d), min(d), max(d),
                     statistics.pstdev(d), statistics.median(d)))
    tot = sum(r[2] for r in rows)
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDev", "MedianNs"])
    for r in sorted(rows, key=lambda r: -r[2]):
        w.writerow([r[0], r[1], r[2], round(r[3], 3), round(100.0 * r[2] / tot, 2), r[4], r[5],
                    round(r[6], 3), r[7]])


if __name__ == "__main__":
    main()
