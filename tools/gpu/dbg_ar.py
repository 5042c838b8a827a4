"""Diagnosis: world-1 all-reduce step vs the exchange-free step at S = 16 --
per-tensor differences of theta and gradients after each of a few steps."""
import os
import sys

import numpy as np

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(R, "distributed-deep-q_amd"))
sys.path.insert(0, R)
import ddq  # noqa: E402
from oracle import ref_numpy as ref  # noqa: E402

S, B, N = 16, 8, 64
rng = np.random.default_rng(2)
nets = [ddq.DeepQNet(batch=B, frame=S) for _ in range(2)]
theta = ref.flatten(ref.init_params(S, seed=9))
st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
for n in nets:
    n.set_flat(0, theta)
    n.set_flat(1, theta)
    n.replay_create(N)
    n.replay_import(st, rng.integers(0, 4, N).astype(np.uint8) * 0,
                    np.zeros(N, np.int16), np.ones(N, np.uint8), 0, N)
uid = ddq.DeepQNet.comm_unique_id()
nets[0].comm_init(uid, 1, 0)
mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
if mode.startswith("test"):   # the test's order: grads set + all-reduced, 3 steps per net
    if mode != "test_nopre":
        g = rng.normal(0, 1, theta.size).astype(np.float32)
        nets[0].set_grads_flat(g)
        nets[0].allreduce_grads()
    for i, n in enumerate(nets):
        cfg = n.step_cfg("sgd", lr=1e-3, target_period=10, allreduce=(i == 0), seed=5)
        if mode == "test_g1":
            for _ in range(3):
                n.step_graph(cfg, 1)
        else:
            n.step_graph(cfg, 3)
        n.synchronize()
for step in range(3 if not mode.startswith("test") else 1):
    for i, n in enumerate(nets if not mode.startswith("test") else []):
        cfg = n.step_cfg("sgd", lr=1e-3, target_period=10, allreduce=(i == 0), seed=5)
        if mode == "graph":
            n.step_graph(cfg, 1)
        else:
            n.step(cfg)
        n.synchronize()
    t0 = nets[0].split(nets[0].get_flat(0), "Q")
    t1 = nets[1].split(nets[1].get_flat(0), "Q")
    g0 = nets[0].split(nets[0].get_grads_flat(), "Q")
    g1 = nets[1].split(nets[1].get_grads_flat(), "Q")
    for k in t0:
        for j in range(2):
            dt = int(np.sum(t0[k][j] != t1[k][j]))
            dg = int(np.sum(g0[k][j] != g1[k][j]))
            if dt or dg:
                print("step %d %s[%d]: theta differs at %d, grad at %d (max |dtheta| %.3g)"
                      % (step, k, j, dt, dg, float(np.max(np.abs(t0[k][j] - t1[k][j])))))
print("done")
