"""Monitoring helpers of barista/netutils.py (reference): per-parameter RMS
norms of data and diff, loss extraction, and the NetLogger files
(loss, <name>.gradnorm, <name>.norm appended per call, netutils.py:72-96)."""
from __future__ import annotations

import os
from datetime import datetime

import numpy as np


def _norms(net, attr, params=None, ord=None):
    p = net.params
    out = {}
    for name in (params or p):
        out[name] = []
        for blob in p[name]:
            a = np.ravel(getattr(blob, attr))
            n = np.linalg.norm(a, ord=ord)
            if ord != 0:
                n /= np.sqrt(a.size)
            out[name].append(n)
    return out


def compute_gradient_norms(net, params=None, ord=None):
    """netutils.py:7-20."""
    return _norms(net, "diff", params, ord)


def compute_param_norms(net, params=None, ord=None):
    """netutils.py:23-36."""
    return _norms(net, "data", params, ord)


def extract_net_data(net, blobs):
    """netutils.py:48-53."""
    b = net.blobs
    return {name: np.squeeze(b[name].data) for name in blobs}


def set_net_params(net, params):
    """netutils.py:61-64: assign {name: [W, b]} into the network."""
    dq = getattr(net, "dqn", net)
    dq.set_params(params)


def pretty_print(param_dict):
    for name in sorted(param_dict):
        print(name.ljust(19), param_dict[name])


class NetLogger:
    def __init__(self, net, path, reset=False):
        self.path = path + "-" + str(datetime.now())
        os.makedirs(self.path, exist_ok=True)
        self.net = net

    def write(self):
        data = extract_net_data(self.net, ("loss",))
        grads = compute_gradient_norms(self.net)
        norms = compute_param_norms(self.net)
        with open(os.path.join(self.path, "loss"), "a") as fp:
            print(data["loss"], file=fp)
        for name, v in grads.items():
            with open(os.path.join(self.path, name + ".gradnorm"), "a") as fp:
                print(",".join(str(x) for x in v), file=fp)
        for name, v in norms.items():
            with open(os.path.join(self.path, name + ".norm"), "a") as fp:
                print(",".join(str(x) for x in v), file=fp)
