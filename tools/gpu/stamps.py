"""Phase stamps of a DDQ_STAMPS variant build (common.h DDQ_STAMP): run a few
eager forward/backward passes at the given frame / batch and print, per stamp
slot, the median time since the workgroup's own slot 0 and since the earliest
slot-0 stamp of the launch (the launch's start).

Usage: DDQ_LIB_PATH=<variant .so> python tools/gpu/stamps.py [S] [B] [reps]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-deep-q_amd"))
import ddq  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
SLOTS, BLOCKS = 48, 512

net = ddq.DeepQNet(batch=B, frame=S)
rng = np.random.default_rng(0)
st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
act = np.eye(4, dtype=np.float32)[rng.integers(0, 4, B)].reshape(B, 4, 1, 1)
net.write_minibatch(st, act, rng.standard_normal((B, 1, 1, 1)).astype(np.float32), ns,
                    np.ones((B, 1, 1, 1), np.float32))
lib = net.lib
lib.ddq_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
buf = np.zeros(SLOTS * BLOCKS, np.uint64)
runs = []
for r in range(reps + 2):
    net.forward_backward()
    assert lib.ddq_debug_stamps(buf.ctypes.data, buf.size) == 0
    if r >= 2:
        runs.append(buf.reshape(BLOCKS, SLOTS).astype(np.int64).copy())
for r, t in enumerate(runs):
    # kernels stamp disjoint slot ranges (small.h: K1 0..7, K3 8..15, K2
    # 16..23, K4 conv2 tiles 24..31, conv3 tiles 32..39)
    for lo in (0, 8, 16, 24, 32):
        tt = t[t[:, lo] > 0]
        if not len(tt):
            continue
        t0 = tt[:, lo].min()
        used = [k for k in range(lo, lo + 8) if (tt[:, k] > 0).any()]
        rel = {k: (np.median(tt[:, k] - tt[:, lo]) * 10 / 1000, (tt[:, k].max() - t0) * 10 / 1000)
               for k in used}
        print("run %d slots %d+: %d blocks, span %.2f us; slot: median since own start / last "
              "since launch start (us): %s" % (r, lo, len(tt), (tt[:, used].max() - t0) * 10 / 1000,
                                            " ".join("%d:%.2f/%.2f" % (k, a, b) for k, (a, b) in rel.items())))
