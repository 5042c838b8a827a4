"""The two helpers of barista/netutils.py (reference) the worker loop and the
evaluator use.  The reference's norm monitoring and NetLogger files
(netutils.py:7-36, 72-96) are out of scope."""
from __future__ import annotations

import numpy as np


def extract_net_data(net, blobs):
    """netutils.py:48-53: squeezed copies of the named blobs."""
    b = net.blobs
    return {name: np.squeeze(b[name].data) for name in blobs}


def set_net_params(net, params):
    """netutils.py:61-64: assign {name: [W, b]} into the network."""
    dq = getattr(net, "dqn", net)
    dq.set_params(params)
