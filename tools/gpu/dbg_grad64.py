"""Debug: fc4 gradient block after exchange-free steps at S = 16 / 64."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-deep-q_amd"))
import numpy as np
import ddq
from ddq.params import init_params_flat
for S in (16, 64):
    B, N = 32, 300
    rng = np.random.default_rng(41)
    theta = init_params_flat(S, seed=42)
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    acts = rng.integers(0, 4, N).astype(np.uint8)
    rws = rng.integers(-1, 2, N).astype(np.int16)
    nts = (rng.random(N) > 0.1).astype(np.uint8)
    n = ddq.DeepQNet(batch=B, frame=S)
    n.set_flat(0, theta); n.set_flat(1, theta)
    n.replay_create(N); n.replay_import(st, acts, rws, nts, 0, N)
    cfg = n.step_cfg("rmsprop", lr=1e-4, target_period=3, seed=4)
    _, o, c = n.layout["Qfc4"][0]
    for what, run in (("eager", lambda: n.step(cfg)), ("pipelined", lambda: n.step_pipelined(cfg, 9)),
                      ("graph", lambda: n.step_graph(cfg, 5))):
        th0 = n.get_flat(0)
        run()
        n.synchronize()
        g = n.get_grads_flat(); th = n.get_flat(0)
        print(S, what, "fc4 grad nnz %d/%d" % (np.count_nonzero(g[o:o + c]), c),
              "fc4 theta changed %d" % np.count_nonzero(th[o:o + c] != th0[o:o + c]),
              "all grad nnz %d" % np.count_nonzero(g), "loss", float(n.blob("loss")), flush=True)
    loss = n.forward_backward()
    g2 = n.get_grads_flat()
    print(S, "full_pass loss", loss, "fc4 grad nnz", np.count_nonzero(g2[o:o + c]), flush=True)
    n.close()
