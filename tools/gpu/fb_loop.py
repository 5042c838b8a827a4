"""Eager forward/backward passes at a frame / batch, for kernel traces of a
variant build: DDQ_LIB_PATH=<.so> rocprofv3 --kernel-trace --stats -- python3
tools/gpu/fb_loop.py [S] [B] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-deep-q_amd"))
import ddq  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
net = ddq.DeepQNet(batch=B, frame=S)
rng = np.random.default_rng(0)
st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
act = np.eye(4, dtype=np.float32)[rng.integers(0, 4, B)].reshape(B, 4, 1, 1)
net.write_minibatch(st, act, rng.standard_normal((B, 1, 1, 1)).astype(np.float32), ns,
                    np.ones((B, 1, 1, 1), np.float32))
for _ in range(reps):
    net.forward_backward()
net.synchronize()
print("done")
