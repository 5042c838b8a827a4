"""Host-side breakdown of the C5 ticket loop at world size 1 (ddq/dist.py
AsyncTicketLoop): per tick, the time spent waiting for readiness, in store
operations and in the ddq_async_tick enqueue, against the device step time.

usage: python tools/gpu/ticket_prof.py [S] [ticks]"""
import os
import sys
import time

import numpy as np

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(R, "distributed-deep-q_amd"))
sys.path.insert(0, R)
import bench  # noqa: E402
from ddq import dist as ddist  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T = int(sys.argv[2]) if len(sys.argv) > 2 else 400
net = bench.make_net(32, S, 30000, 0, 0)
net.comm_init(net.comm_unique_id(), 1, 0)
cfg = net.step_cfg("rmsprop", lr=1e-4, target_period=10, exchange="async", seed=1234)
store = ddist.ticket_store(1, 0)
loop = ddist.AsyncTicketLoop(net, cfg, store, 0, 1)
loop.run(20)
net.synchronize()
t0 = time.perf_counter()
loop.run(T)
net.synchronize()
dt = (time.perf_counter() - t0) / T
# the parts, timed by hand on the same loop's primitives
ready, ops, tick = [], [], []
net.async_begin(cfg)
for _ in range(100):
    a = time.perf_counter()
    while not net.async_ready():
        pass
    b = time.perf_counter()
    t = store.add("x", 1)
    store.set("y/%d" % t, "0")
    store.check(["y/%d" % t])
    store.get("y/%d" % t)
    c = time.perf_counter()
    net.async_tick(cfg, 0)
    d = time.perf_counter()
    ready.append(b - a); ops.append(c - b); tick.append(d - c)
net.synchronize()
print("ticket loop: %.1f us per tick (%.0f ticks/s)" % (dt * 1e6, 1 / dt))
print("busy-wait for readiness: median %.1f us; 4 store ops: %.1f us; async_tick enqueue: %.1f us"
      % (np.median(ready) * 1e6, np.median(ops) * 1e6, np.median(tick) * 1e6))

