"""A/B of deepq16 step throughput between library builds (DDQ_LIB_PATH per
run, fresh processes, alternating): bench.py deepq16_line (S = 16, B = 32,
pipelined 8-step graphs, rmsprop with the fused apply).
usage: python tools/gpu/ab16.py <lib-or-'prod'> <lib-or-'prod'> [rounds] [steps]"""
import json
import os
import subprocess
import sys

libs = sys.argv[1:3]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3000
code = ("import sys, json; sys.path.insert(0, '.'); import bench; "
        "r = bench.deepq16_line(steps=%d); print(json.dumps({k: r[k] for k in "
        "('updates_per_s', 'kernels_us')}))" % steps)
res = {l: [] for l in libs}
for i in range(rounds):
    for l in libs:
        env = dict(os.environ)
        env.pop("DDQ_LIB_PATH", None)
        if l != "prod":
            env["DDQ_LIB_PATH"] = os.path.abspath(l)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                             timeout=300)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        r = json.loads(line[-1]) if line else {"error": out.stderr[-400:]}
        res[l].append(r)
        print(i, l, json.dumps(r), flush=True)
for l in libs:
    v = [r["updates_per_s"] for r in res[l] if "updates_per_s" in r]
    print("%s: updates/s %s median %.1f" % (l, v, sorted(v)[len(v) // 2] if v else 0), flush=True)
