"""Summarise rocprofv3 counter_collection CSVs: per kernel, mean counter value per dispatch."""
import csv, glob, os, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
def short(n):
    for key in ("ConvFwd", "ConvWgrad", "ConvDgrad", "FcFwd", "FcDgrad", "FcWgrad"):
        if key in n:
            i = n.index(key); return n[i:i + 40].split(">")[0] + ("" if "gemm" not in n else "[gemm]")
    if "direct_conv_kernel" in n:
        return "direct<" + n.split("direct_conv_kernel<")[1].split(">")[0] + ">"
    return n.split("(")[0][-40:]
cols = ["FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
        "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT",
        "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE"]
print("kernel".ljust(46) + "".join(c[-14:].rjust(15) for c in cols))
for name, d in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("GRBM_GUI_ACTIVE", [0]))):
    row = short(name).ljust(46)
    for c in cols:
        v = d.get(c)
        row += ("%.4g" % (sum(v) / len(v)) if v else "-").rjust(15)
    print(row)
