"""World-size-2 gloo tests (CPU) of the multi-GPU path's host logic:
communicator-id bootstrap, per-rank index streams, max-over-ranks timing, and
the sync-DP semantics (sum of W gradients at the same theta, applied once ==
the reference server applying W equally-stale SGD gradients in sequence).
The per-rank gradients come from the oracle (checker), the collective from
torch.distributed's gloo all_reduce -- the same sum RCCL performs on GPU."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "distributed-deep-q_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ddq import dist as ddist
    from oracle import ref_numpy as ref
    ddist.init_process_group(rank, world, "gloo")
    # 1) unique id: rank 0's bytes reach every rank
    uid = ddist.broadcast_unique_id(rank, lambda: bytes(range(128)))
    # 2) per-rank gradient on this rank's own minibatch, same theta
    S, B = 16, 2
    theta = ref.flatten(ref.init_params(S, seed=1))
    rng = np.random.default_rng(ddist.index_seed(1234, rank))
    st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    act = np.zeros((B, 4, 1, 1), np.float32)
    act[np.arange(B), rng.integers(0, 4, B)] = 1
    rw = rng.integers(-1, 2, (B, 1, 1, 1)).astype(np.float32)
    nt = np.ones((B, 1, 1, 1), np.float32)
    pq = ref.unflatten(theta, S, "Q")
    pp = ref.unflatten(theta, S, "P")
    _, g = ref.full_pass(pq, pp, st, act, rw, ns, nt)
    g = ref.flatten(g).astype(np.float32)
    t = torch.from_numpy(g.copy())
    dist.all_reduce(t)                       # the sync-DP exchange (sum)
    theta_dp = ref.sgd_update(theta, t.numpy(), 1e-3)
    gathered = [torch.zeros_like(torch.from_numpy(g)) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(g))
    # reference server: apply each worker's gradient on arrival (same theta)
    theta_ps = theta.copy()
    for gi in gathered:
        theta_ps = ref.sgd_update(theta_ps, gi.numpy(), 1e-3)
    tmax = ddist.max_over_ranks(float(rank + 1))
    out.put((rank, uid, np.abs(theta_dp - theta_ps).max(), np.abs(theta_dp - theta).max(),
             tmax, int(rng.integers(0, 1 << 30))))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gloo_sync_dp_semantics():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, uid0, d0, m0, t0, s0), (r1, uid1, d1, m1, t1, s1) = res
    assert uid0 == uid1 == bytes(range(128))
    # sum-then-apply == sequential SGD up to fp32 rounding (a few ulp of theta)
    assert d0 < 1e-8 + 1e-3 * m0 and d1 < 1e-8 + 1e-3 * m1
    assert m0 > 0
    assert t0 == t1 == 2.0                    # max over ranks
    assert s0 != s1                           # distinct per-rank index streams
