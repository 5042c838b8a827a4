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


def _shard_len(P, W):
    """Shard geometry of ddq_comm_init / ddq_group_init (api.hip setup_shards)."""
    return ((P + W * 64 - 1) // (W * 64)) * 64


def _exchange_worker(rank, world, port, out):
    """The SERVER and SHARDED exchanges restated over gloo with the library's
    shard geometry: gradient slices to their owners (all-gather + slicing
    stands in for RCCL's all-to-all / reduce-scatter), the owner applies its
    slice (W gradients one by one in rank order, or their sum), then the
    owners' shards are all-gathered into every replica."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "distributed-deep-q_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ddq import dist as ddist
    from oracle import ref_numpy as ref
    ddist.init_process_group(rank, world, "gloo")
    S = 16
    P = ref.num_params(S)
    L = _shard_len(P, world)
    theta = ref.flatten(ref.init_params(S, seed=3))
    rng = np.random.default_rng(100 + rank)
    g = rng.normal(0, 1e-2, P).astype(np.float32)
    gp = np.zeros(world * L, np.float32)
    gp[:P] = g
    allg = [torch.zeros(world * L) for _ in range(world)]
    dist.all_gather(allg, torch.from_numpy(gp))
    mine = slice(rank * L, (rank + 1) * L)
    th = np.zeros(world * L, np.float32)
    th[:P] = theta
    res = {}
    for mode in ("server", "sharded"):
        shard, cache = th[mine].copy(), None
        slices = [a.numpy()[mine] for a in allg]        # what the all-to-all delivers
        if mode == "server":
            for s in slices:                           # ticket (rank) order
                shard, cache = ref.rmsprop_update(shard, s, cache, 1e-3)
        else:
            shard, cache = ref.rmsprop_update(shard, np.sum(slices, axis=0,
                                                            dtype=np.float32), None, 1e-3)
        parts = [torch.zeros(L) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(shard)))
        res[mode] = torch.cat(parts).numpy()[:P]
    out.put((rank, res["server"], res["sharded"],
             np.stack([a.numpy()[:P] for a in allg])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_server_and_sharded_exchange_semantics(world):
    """Every replica ends with the same theta, equal to the param server
    applying the W gradients on arrival in rank order (server.py:196-209,
    rmsprop lagged cache across them) resp. applying their sum once; shards
    of ceil(P/(64W))*64 cover P for W not dividing P."""
    from oracle import ref_numpy as ref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    S = 16
    theta = ref.flatten(ref.init_params(S, seed=3))
    grads = res[0][3]
    want_srv, cache = theta.copy(), None
    for g in grads:
        want_srv, cache = ref.rmsprop_update(want_srv, g, cache, 1e-3)
    want_sh, _ = ref.rmsprop_update(theta, grads.sum(axis=0, dtype=np.float32), None, 1e-3)
    for r, srv, sh, _ in res:
        np.testing.assert_array_equal(srv, res[0][1])
        np.testing.assert_array_equal(sh, res[0][2])
        np.testing.assert_allclose(srv, want_srv, rtol=0, atol=1e-6)
        np.testing.assert_allclose(sh, want_sh, rtol=0, atol=1e-6)
    # the two semantics differ (rmsprop: W lagged applies != one summed apply)
    assert np.abs(res[0][1] - res[0][2]).max() > 1e-5


def _mode_worker(rank, world, port, fail, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "distributed-deep-q_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ddq import dist as ddist
    from ddq._lib import DDQError
    ddist.init_process_group(rank, world, "gloo")

    class Cfg:
        overlap = 0

    class FakeNet:   # step_prepare refuses the modes listed for this rank
        def step_prepare(self, cfg, mode):
            if (mode, bool(cfg.overlap)) in fail.get(rank, ()):
                raise DDQError(-3, "capture refused on rank %d" % rank)

    modes = [("pipelined", True), ("graph", False), ("eager", False)]
    out.put((rank, ddist.choose_step_mode(FakeNet(), Cfg(), modes)))
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.parametrize("fail,want", [({}, ("pipelined", True)),
                                       ({1: {("pipelined", True)}}, ("graph", False)),
                                       ({0: {("pipelined", True)}, 2: {("graph", False)}},
                                        ("eager", False))])
def test_step_mode_fallback_is_collective(fail, want):
    """bench.py's graph-capture fallback: one rank failing to prepare a mode
    moves EVERY rank to the next mode (no rank left waiting in a collective)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_mode_worker, args=(r, world, port, fail, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(res[r] == want for r in range(world)), res
