"""Print the headline fields of a bench.py JSON line (file argument)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("bench", d["value"], d["ms_per_step"], d.get("step_ms_distribution"))
print("roofline", {k: d["roofline"].get(k) for k in ("kernel", "frac", "kernel_us", "step_frac",
                                                     "step_ideal_us", "traffic")})
print("kernels", json.dumps(d["kernels_us"]))
for k, v in d.get("exchange_paths", {}).get("paths", {}).items():
    print("exchange", k, v["updates_per_s"], v["vs_exchange_free"], v["mode"])
if "deepq16" in d:
    print("deepq16", d["deepq16"])
if "frame_sweep" in d:
    print("sweep", [(f["frame"], f["updates_per_s"], f["frac_of_step_roofline"])
                    for f in d["frame_sweep"]["frames"]])
if "cpu_baseline" in d:
    c = d["cpu_baseline"]
    print("cpu", c["value"], c["cores"], c["single_core"]["value"],
          [(e["batch"], e["frame"], e["value"], e["single_core"]["value"]) for e in c.get("configs", [])])
if "gather_stress" in d:
    print("gather", [(e["n"], e["gather_GBps"], e["frac"]) for e in d["gather_stress"]["launches"]])
