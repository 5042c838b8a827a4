"""Summarise a rocprofv3 kernel-trace directory: median device time of each
step kernel over the graph-replayed steps, plus the bench JSON value.

Usage: python tools/trace_summary.py <rocprof out dir> [label]"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

SHORT = [("sample_gather_kernel", "sample"), ("split_conv1_kernel", "c1f"),
         ("c2f", "c2f"), ("c3f", "c3f"), ("c3d", "c3d"), ("c2d", "c2d"),
         ("wgrads_pair_kernel", "c23w"),
         ("wgrads_kernel<64, 64, 3", "c3w"), ("wgrads_kernel<32, 64, 5", "c2w"),
         ("wgrad1s_kernel", "c1w"),
         ("fc4_fwd_split", "fc4f"), ("fc4_head", "head"), ("fc4_bwd_kernel", "fc4bwd"),
         ("wgrad_reduce_kernel", "wred"), ("apply_kernel", "apply")]
# split_conv_kernel<CPT, CP, N, KS, ..., DGRAD>: any tile of the per-map menus
SPLIT = {(32, 64, 5, "false"): "c2f", (64, 64, 3, "false"): "c3f", (64, 64, 3, "true"): "c3d",
         (64, 32, 5, "true"): "c2d"}


def main():
    d = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        m = re.search(r"split_conv_kernel<(\d+), \d+, (\d+), (\d+),.*(true|false)(, \d+)*>", name)
        if m:
            short = SPLIT.get((int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(4)))
            if short:
                per[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            continue
        for key, short in SHORT:
            if key in name:
                per[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                break
    out = {k: round(statistics.median(v), 2) for k, v in per.items() if v}
    tot = sum(out.values())
    js = d.rstrip("/") + ".json"
    val = ""
    if os.path.exists(js):
        try:
            b = json.load(open(js))
            val = "%s upd/s %.4f ms" % (b["value"], b["ms_per_step"])
        except Exception:
            pass
    print("variant %s: %s | sum %.1f us | %s" % (label, val, tot,
          " ".join("%s=%.1f" % (k, out[k]) for k in dict.fromkeys(k for _, k in SHORT) if k in out)))


if __name__ == "__main__":
    main()
