"""Debug: per-step comparison of the shipped step path with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-deep-q_amd"), os.path.join(ROOT, "tests")]
import ddq  # noqa: E402
from ddq.expgain import synthetic_transitions  # noqa: E402
from ddq.params import init_params_flat  # noqa: E402
from oracle import ref_numpy as ref  # noqa: E402

S, B, N = int(os.environ.get("S", 64)), 32, 30000
mode = sys.argv[1] if len(sys.argv) > 1 else "pipelined"
pool = 4096
st, ac, rw, nt = synthetic_transitions(pool, S, seed=1000)
reps = (N + pool - 1) // pool
st, ac, rw, nt = (np.tile(st, (reps, 1, 1, 1))[:N], np.tile(ac, reps)[:N], np.tile(rw, reps)[:N],
                  np.tile(nt, reps)[:N])
theta = init_params_flat(S, seed=42)
net = ddq.DeepQNet(batch=B, frame=S)
net.set_flat(0, theta)
net.set_flat(1, theta)
net.replay_create(N)
net.replay_import(st, ac, rw, nt.astype(np.uint8), 0, N)
net.index_log_enable(64)
cfg = net.step_cfg("rmsprop", lr=1e-4, target_period=10, seed=1234)
r = ref.ReplayRef((4, S, S), N)
r.state, r.action, r.reward, r.non_terminal = st, ac, rw, nt.astype(bool)
r.head, r.valid = 0, N
thq = theta.copy()
thp = theta.copy()
state = None
d0 = net.replay_draws()
for t in range(int(os.environ.get("T", 4))):
    if mode == "pipelined":
        net.step_pipelined(cfg, 1)
    elif mode == "graph":
        net.step_graph(cfg, 1)
    else:
        net.step(cfg)
    net.synchronize()
    idx = net.index_log(d0 + t, 1)[0]
    print("step", t, "idx", idx[:6], "read_indices", net.read_indices()[:6])
    if t % 10 == 0:
        thp = thq.copy()
    mb = r.gather(idx)
    gmb = net.read_minibatch()
    for a, b_, nm in zip(gmb, mb, ["state", "action", "reward", "next", "nt"]):
        if not np.array_equal(np.asarray(a).ravel(), np.asarray(b_).ravel()):
            print("  minibatch mismatch", nm)
    blobs, grads = ref.full_pass(ref.unflatten(thq, S, "Q"), ref.unflatten(thp, S, "P"), *mb)
    g = ref.flatten(grads).astype(np.float32)
    gg = net.get_grads_flat()
    print("  loss gpu %.6g ref %.6g" % (float(net.blob("loss")), blobs["loss"]))
    print("  grad max abs err %.3g scale %.3g" % (np.abs(gg - g).max(), np.abs(g).max()))
    thq, state = ref.rmsprop_update(thq, g, state, 1e-4, 0.9)
    gq = net.get_flat(0)
    e = np.abs(gq - thq)
    print("  theta max abs err %.3g (at %d) changed %.3g" % (e.max(), e.argmax(), np.abs(thq - theta).max()))
    c = net.optimizer_state()
    print("  cache max abs err %.3g scale %.3g" % (np.abs(c - state).max(), np.abs(state).max()))
