"""Debug: per-layer routing mismatches GPU vs oracle over frame sizes."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-deep-q_amd")]
import numpy as np
import ddq
from oracle import ref_numpy as ref
for S, B in [(16, 8), (32, 8), (48, 4), (64, 4), (64, 32)]:
    rng = np.random.default_rng(1)
    pQ = ref.init_params(S, seed=7, prefix="Q"); pP = ref.init_params(S, seed=8, prefix="P")
    for p in (pQ, pP):
        for k in p:
            p[k][0] = (p[k][0] * 3).astype(np.float32)
    net = ddq.DeepQNet(batch=B, frame=S)
    d = dict(pQ); d.update(pP); net.set_params(d)
    st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    act = np.zeros((B, 4), np.float32); act[:, 0] = 1
    net.write_minibatch(st, act, np.zeros(B, np.float32), ns, np.ones(B, np.float32))
    net.forward_backward()
    blobs, grads, cache = ref.full_pass(pQ, pP, st, act.reshape(B, 4, 1, 1), np.zeros((B, 1, 1, 1)), ns, np.ones((B, 1, 1, 1)), return_cache=True)
    qo = net.blob("Q_out").reshape(B, 4)
    print("S=%d B=%d Q_out maxrel %.3g" % (S, B, np.abs(qo - blobs["Q_out"]).max() / np.abs(blobs["Q_out"]).max()))
    for i in (1, 2, 3):
        g = net.pool_mask(i); r = ref.route_codes(cache["act%d" % i], cache["arg%d" % i])
        bad = np.argwhere(g != r)
        print("  layer", i, "mismatch", len(bad), "of", g.size, bad[:3].tolist(), (g[tuple(bad[0])], r[tuple(bad[0])]) if len(bad) else "")
    net.close()
