"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv.

Usage: python tools/timeline.py <kernel_trace.csv> [--step-kernel apply_kernel] [--nsteps 3]
Prints, for a few consecutive steps in the middle of the trace, every kernel's
start offset from the step start, its duration and the idle gap before it on
the device (all streams merged), plus per-step totals.
"""
import csv
import sys


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "ddq::"):
        n = n.replace(pre, "")
    return n[:70]


def main():
    path = sys.argv[1]
    marker = "apply_kernel"
    nsteps = 3
    if "--step-kernel" in sys.argv:
        marker = sys.argv[sys.argv.index("--step-kernel") + 1]
    if "--nsteps" in sys.argv:
        nsteps = int(sys.argv[sys.argv.index("--nsteps") + 1])
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in rows), key=lambda t: t[0])
    ends = [i for i, k in enumerate(ks) if marker in k[2]]
    if len(ends) < nsteps + 2:
        print("not enough steps"); return
    mid = len(ends) // 2
    for s in range(mid, mid + nsteps):
        lo, hi = ends[s - 1] + 1, ends[s]
        t0 = ks[lo][0]
        busy_end = ks[lo - 1][1]
        print("---- step (%d kernels), wall %.1f us" % (hi - lo + 1, (ks[hi][1] - ks[lo - 1][1]) / 1e3))
        idle = 0
        for s0, e0, n in ks[lo:hi + 1]:
            gap = max(0, s0 - busy_end)
            idle += gap
            busy_end = max(busy_end, e0)
            print("  %8.1f  %7.1f  gap %5.1f  %s" % ((s0 - t0) / 1e3, (e0 - s0) / 1e3, gap / 1e3, short(n)))
        print("  device idle inside step: %.1f us" % (idle / 1e3))


if __name__ == "__main__":
    main()
