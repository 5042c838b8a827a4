"""Full-pass parity diagnosis: every blob / gradient tensor's worst error
against the oracle as a multiple of the tolerance (tests/_parity.py), without
stopping at the first failure.  Usage: python tools/gpu/dbg_parity.py S B frames init"""
import os
import sys

import numpy as np

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "distributed-deep-q_amd"))
sys.path.insert(0, R)
import ddq  # noqa: E402
from oracle import ref_numpy as ref  # noqa: E402
from _parity import full_pass_gpu_routing, RTOL, COND  # noqa: E402
from test_gpu_parity import make_inputs, make_params  # noqa: E402

S, B = int(sys.argv[1]), int(sys.argv[2])
frames, init = sys.argv[3], sys.argv[4]
rng = np.random.default_rng(100 + S + B)
pQ, pP = make_params(ref, rng, S, init)
net = ddq.DeepQNet(batch=B, frame=S)
params = dict(pQ)
params.update(pP)
net.set_params(params)
mb = make_inputs(rng, B, S, frames)
net.write_minibatch(*mb)
net.forward_backward()
blobs, grads, nties = full_pass_gpu_routing(ref, net, pQ, pP, mb)
routes = {i: net.pool_mask(i) for i in (1, 2, 3)}
mblobs, mgrads = ref.magnitudes(pQ, pP, *mb, routes=routes)
print("near ties", nties)


def rep(what, g, r, m):
    g = np.asarray(g, np.float64).reshape(r.shape)
    err = np.abs(g - r)
    tol = RTOL * np.abs(r) + COND * m + 1e-30
    q = err / tol
    i = np.unravel_index(np.argmax(q), r.shape)
    print("%-12s worst err/tol %.3g at %s (gpu %.6g ref %.6g |terms| %.3g), n over %d/%d, max err/M %.3g"
          % (what, q[i], i, g[i], r[i], m[i], int((q > 1).sum()), r.size, float(np.max(err / (m + 1e-300)))))


for name, shape in (("Q_out", (B, 4)), ("P_out", (B, 4)), ("Q_sa", (B,)), ("target_Q_sa", (B,))):
    rep(name, net.blob(name).reshape(shape), np.asarray(blobs[name]), np.asarray(mblobs[name]))
g = net.split(net.get_grads_flat(), "Q")
for name in grads:
    for i in range(2):
        rep("%s[%d]" % (name, i), g[name][i], np.asarray(grads[name][i]), np.asarray(mgrads[name][i]))
