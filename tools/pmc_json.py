"""Per-kernel PMC means from rocprofv3 counter_collection CSVs -> JSON.

HBM bytes per dispatch follow MI355X_MICROARCH.md (HBM [CDNA4]): FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced read, so fetch_bytes = 2 * 1024 * FETCH_SIZE; write_bytes =
1024 * WRITE_SIZE.  Each counter comes from its own pass (tools/pmc_passes.txt).

usage: python tools/pmc_json.py <rocprof pmc dir> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root, out = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r.get("Kernel_Name", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for name, d in acc.items():
        m = {k: sum(v) / len(v) for k, v in d.items()}
        e = {"dispatches": max(len(v) for v in d.values()), "counters": m}
        if "FETCH_SIZE" in m:
            e["fetch_bytes"] = 2.0 * 1024.0 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            e["write_bytes"] = 1024.0 * m["WRITE_SIZE"]
        if "fetch_bytes" in e and "write_bytes" in e:
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        res[name] = e
    json.dump({"source": root, "correction": "fetch x2 (gfx950), KiB->bytes", "kernels": res},
              open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
