"""Debug: pipelined chain vs eager steps, bit-exactness by chain length."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-deep-q_amd")]
import ddq  # noqa: E402
from ddq.expgain import synthetic_transitions  # noqa: E402
from ddq.params import init_params_flat  # noqa: E402

S, B, N = int(os.environ.get("S", 64)), 32, 30000
pool = 4096
st, ac, rw, nt = synthetic_transitions(pool, S, seed=1000)
reps = (N + pool - 1) // pool
st, ac, rw, nt = (np.tile(st, (reps, 1, 1, 1))[:N], np.tile(ac, reps)[:N], np.tile(rw, reps)[:N],
                  np.tile(nt, reps)[:N])
theta = init_params_flat(S, seed=42)


def mk():
    net = ddq.DeepQNet(batch=B, frame=S)
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    net.replay_create(N)
    net.replay_import(st, ac, rw, nt.astype(np.uint8), 0, N)
    net.index_log_enable(64)
    return net


for k in [int(x) for x in sys.argv[1:]]:
    for mode in ("pipelined", "graph"):
        a, b = mk(), mk()
        cfg = a.step_cfg("rmsprop", lr=1e-4, target_period=10, seed=1234)
        if mode == "pipelined":
            a.step_pipelined(cfg, k)
        else:
            a.step_graph(cfg, k)
        for _ in range(k):
            b.step(cfg)
        a.synchronize()
        b.synchronize()
        la, lb = a.index_log(0, k), b.index_log(0, k)
        same_idx = np.array_equal(la, lb)
        ta, tb = a.get_flat(0), b.get_flat(0)
        pa, pb = a.get_flat(1), b.get_flat(1)
        print("k=%d %s: idx same %s, thetaQ max diff %.3g, thetaP max diff %.3g, opt diff %.3g"
              % (k, mode, same_idx, np.abs(ta - tb).max(), np.abs(pa - pb).max(),
                 np.abs(a.optimizer_state() - b.optimizer_state()).max()))
        if not same_idx:
            bad = [i for i in range(k) if not np.array_equal(la[i], lb[i])]
            print("   first differing draw", bad[:5], la[bad[0]][:6], lb[bad[0]][:6])
        a.close()
        b.close()
