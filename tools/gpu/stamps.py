"""Phase stamps of a DDQ_STAMPS variant build (common.h DDQ_STAMP): run a few
eager forward/backward passes at the given frame / batch and print, per stamp
slot, the median time since the workgroup's own slot 0 and since the earliest
slot-0 stamp of the launch (the launch's start).

Usage: DDQ_LIB_PATH=<variant .so> python tools/gpu/stamps.py [S] [B] [reps] [fb|step]
("step": the bench's pipelined graph step, rmsprop with the fused apply)"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-deep-q_amd"))
import ddq  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
mode = sys.argv[4] if len(sys.argv) > 4 else "fb"
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
if mode == "step":
    from ddq.params import init_params_flat
    theta = init_params_flat(S, seed=42)
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    N = 4096
    net.replay_create(N)
    net.replay_import(rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8),
                      rng.integers(0, 4, N).astype(np.uint8), rng.integers(-1, 2, N).astype(np.int16),
                      (rng.random(N) > 0.05).astype(np.uint8), 0, N)
    cfg = net.step_cfg("rmsprop", lr=1e-4, target_period=10, seed=1234)
    net.step_prepare(cfg, "pipelined")
    net.step_pipelined(cfg, 20)
for r in range(reps + 2):
    if mode == "step":
        net.step_pipelined(cfg, 1)
        net.synchronize()
    else:
        net.forward_backward()
    assert lib.ddq_debug_stamps(buf.ctypes.data, buf.size) == 0
    if r >= 2:
        runs.append(buf.reshape(BLOCKS, SLOTS).astype(np.int64).copy())
for r, t in enumerate(runs):
    # kernels stamp disjoint slot ranges (small.h: K1 0..7, K3 8..15, K2
    # 16..23, K4 conv2 tiles 24..31, conv3 tiles 32..39)
    for lo in (0, 8, 16, 24, 32, 40, 42):
        tt = t[t[:, lo] > 0]
        if not len(tt):
            continue
        t0 = tt[:, lo].min()
        seq = [16, 17, 18, 19, 20, 44, 45, 46, 21, 22, 23] if lo == 16 else \
            ([lo, lo + 1, lo + 2, lo + 3, lo + 4, lo + 6, lo + 5] if lo in (24, 32) else
             range(lo, lo + (2 if lo >= 40 else 8)))
        used = [k for k in seq if (tt[:, k] > 0).any()]
        # each slot over the workgroups that wrote it (K2's P-tower workgroups
        # leave after slot 18; an unwritten slot is 0, not a time)
        rel = {}
        for k in used:
            w = tt[tt[:, k] > 0]
            rel[k] = (np.median(w[:, k] - w[:, lo]) * 10 / 1000, (w[:, k].max() - t0) * 10 / 1000)
        print("run %d slots %d+: %d blocks, span %.2f us; slot: median since own start / last "
              "since launch start (us): %s" % (r, lo, len(tt), (tt[:, used].max() - t0) * 10 / 1000,
                                            " ".join("%d:%.2f/%.2f" % (k, a, b) for k, (a, b) in rel.items())))
# the meeting tiles' arrival skew: per K4 block (conv2 24.., conv3 32..) the
# pre-meeting stamp since the launch's start, slowest first
for lo, name in ((24, "conv2"), (32, "conv3")):
    t = runs[-1]
    t0 = t[t[:, 16 if lo == 0 else 24] > 0][:, 24].min() if (t[:, 24] > 0).any() else 0
    sel = np.nonzero((t[:, lo] > 0) & (t[:, lo + 3] > 0))[0]
    arr = sorted(((t[b, lo + 3] - t0) * 10 / 1000, b, [(t[b, lo + k] - t[b, lo]) * 10 / 1000 for k in range(1, 6)])
                 for b in sel)[::-1]
    print("%s pre-meeting arrivals (us since launch), slowest 6: %s" % (
        name, "; ".join("blk %d at %.2f (own: %s)" % (b, a, " ".join("%.2f" % x for x in o)) for a, b, o in arr[:6])))
    print("  median %.2f, fastest %.2f" % (arr[len(arr) // 2][0], arr[-1][0]))
