"""Repeat the W = 1 async exchange against plain steps in fresh processes
(tests/test_gpu_async.py _world1_nets): eager rounds, round-robin graphs or
ticket ticks; prints the parameter counts that differ after 4 and 13 pushes.
usage: python tools/gpu/async_repeat.py <runs> eager,graph,ticket"""
import sys, os, subprocess, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "distributed-deep-q_amd")
def once(mode):
    import ddq
    from test_gpu_async import _world1_nets
    period, R = 3, 13
    nets = _world1_nets(ddq, 2)
    a, p = nets
    a.comm_init(ddq.DeepQNet.comm_unique_id(), 1, 0)
    acfg = a.step_cfg("rmsprop", lr=1e-4, target_period=period, exchange="async", seed=9)
    plain = p.step_cfg("rmsprop", lr=1e-4, target_period=period, exchange="none", seed=9)
    res = []
    def cmp(tag, k):
        for _ in range(k): p.step(plain)
        a.synchronize(); p.synchronize()
        d = [int((a.get_flat(z) != p.get_flat(z)).sum()) for z in (0, 1)]
        res.append("%s:%s" % (tag, d))
    if mode == "eager":
        for i in range(R):
            a.step(acfg)
            if i in (3, 12): cmp("r%d" % (i + 1), 4 if i == 3 else 9)
    elif mode == "graph":
        a.step_graph(acfg, 4); cmp("r4", 4)
        a.step_graph(acfg, R - 4); cmp("r13", 9)
    else:
        a.async_begin(acfg)
        for i in range(R):
            while not a.async_ready():
                pass
            a.async_tick(acfg, 0)
            if i in (3, 12): cmp("t%d" % (i + 1), 4 if i == 3 else 9)
    print("RES", mode, " ".join(res), flush=True)
if len(sys.argv) > 2 and sys.argv[1] == "once":
    once(sys.argv[2]); sys.exit(0)
for mode in sys.argv[2].split(","):
    bad = 0
    for i in range(int(sys.argv[1])):
        r = subprocess.run([sys.executable, "-u", __file__, "once", mode], capture_output=True, text=True, timeout=120)
        line = [l for l in r.stdout.splitlines() if l.startswith("RES")]
        s = line[0] if line else "rc %d %s" % (r.returncode, r.stderr[-300:])
        if s.count("[0, 0]") != 2:
            bad += 1
            print(i, s, flush=True)
    print("mode %s: %d bad of %s" % (mode, bad, sys.argv[1]), flush=True)
