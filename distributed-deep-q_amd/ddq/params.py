"""Parameter layout and initial fillers of the deepq network.

Layout = pycaffe ``net.params`` order of models/deepq/train_val.prototxt
(Qconv1, Qconv2, Qconv3, Qfc4, Q_out; each [weight, bias]) with Caffe-2014
4-D blob shapes; the P tower repeats it with prefix 'P'.  Fillers
(train_val.prototxt:52-59, 92-99, 132-139, 170-177, 206-213): gaussian
std 0.01 (conv, Q_out), 0.005 (fc4), constant-0 biases.  Caffe's RNG stream
cannot be reproduced, so the initial values are seeded numpy draws
(SURVEY.md 8(a) A21); the server copies Q into P at iteration 0
(server.py:188-189).
"""
from __future__ import annotations

import collections

import numpy as np

_CONVS = (("conv1", 32, 7), ("conv2", 64, 5), ("conv3", 64, 3))
_STD = {"conv1": 0.01, "conv2": 0.01, "conv3": 0.01, "fc4": 0.005, "_out": 0.01}


def param_shapes(S, prefix="Q"):
    if S % 8:
        raise ValueError("frame side must be a multiple of 8")
    s4 = S // 8
    out = collections.OrderedDict()
    cin = 4
    for name, cout, k in _CONVS:
        out[prefix + name] = [(cout, cin, k, k), (1, 1, 1, cout)]
        cin = cout
    out[prefix + "fc4"] = [(1, 1, 512, 64 * s4 * s4), (1, 1, 1, 512)]
    out[prefix + "_out"] = [(1, 1, 4, 512), (1, 1, 1, 4)]
    return out


def num_params(S):
    return sum(int(np.prod(s)) for v in param_shapes(S).values() for s in v)


def init_params(S, seed=42, prefix="Q"):
    rng = np.random.default_rng(seed)
    out = collections.OrderedDict()
    for name, (ws, bs) in param_shapes(S, prefix).items():
        out[name] = [rng.normal(0.0, _STD[name[1:]], ws).astype(np.float32),
                     np.zeros(bs, np.float32)]
    return out


def init_params_flat(S, seed=42):
    return np.concatenate([b.ravel() for v in init_params(S, seed).values() for b in v])
