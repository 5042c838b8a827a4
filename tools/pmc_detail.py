"""Per-kernel SQ counter breakdown from several rocprofv3 --pmc passes
(tools/gpu/run.sh PMC=...): mean per dispatch, then derived per-wave shares.

Usage: python tools/pmc_detail.py <pass dir> [<pass dir> ...]"""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    m = re.search(r"direct_conv_kernel<([^>]*)>", n)
    if m:
        return "direct<" + m.group(1) + ">"
    for key in ("wgradd_kernel<", "wgrad1_kernel", "fc4_", "apply_kernel", "wgrad_reduce",
                "sample_gather", "gemm_f32_kernel"):
        if key in n:
            i = n.index(key)
            return n[i:i + 40].split("(")[0]
    return n.split("(")[0][-40:]


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                acc[short(r.get("Kernel_Name", ""))][r["Counter_Name"]].append(
                    float(r["Counter_Value"]))
    mean = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
    print("%-48s %9s %7s %7s %7s %7s %7s %7s %7s %7s %7s" % (
        "kernel", "wavecyc/w", "lvl", "wait%", "wLDS%", "valu%", "lds%", "vmem%", "sca%",
        "misc%", "mfma%"))
    for k, m in sorted(mean.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = m.get("SQ_WAVE_CYCLES", 0)
        if not wc:
            continue
        w = max(m.get("SQ_WAVES", 1), 1)
        pct = lambda c: 100.0 * m.get(c, 0) / wc
        busy = m.get("SQ_BUSY_CYCLES", 0)
        lvl = m.get("SQ_LEVEL_WAVES", 0) / busy if busy else 0
        mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        print("%-48s %9.0f %7.2f %7.1f %7.1f %7.1f %7.1f %7.1f %7.1f %7.1f %7.1f" % (
            k[:48], wc / w, lvl, pct("SQ_WAIT_ANY"), pct("SQ_WAIT_INST_LDS"),
            pct("SQ_ACTIVE_INST_VALU"), pct("SQ_ACTIVE_INST_LDS"), pct("SQ_ACTIVE_INST_VMEM"),
            pct("SQ_ACTIVE_INST_SCA"), pct("SQ_ACTIVE_INST_MISC"), 100.0 * mf / wc))
    print()
    print("raw means per dispatch:")
    cols = sorted({c for m in mean.values() for c in m})
    for k, m in mean.items():
        print(k[:60], {c: "%.4g" % m[c] for c in cols if c in m})


if __name__ == "__main__":
    main()
