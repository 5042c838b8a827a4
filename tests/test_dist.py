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


def _fake_grad(theta, w, k):
    """A deterministic gradient of worker w's k-th minibatch at theta."""
    rng = np.random.default_rng(1000 * w + k)
    return (np.sin(theta * (w + 1)) * 1e-2 + rng.normal(0, 1e-3, theta.size)).astype(np.float32)


def _async_worker(rank, world, port, rounds, period, out):
    """DDQ_EXCHANGE_ASYNC's round-robin schedule (api.hip rccl_async_round)
    restated over gloo point-to-point: at tick w worker w sends its gradient
    slices to the owners, each owner applies its slice to its shard of the
    central model on arrival (rmsprop, lagged cache), the central P shard
    follows Q when the tick's iteration is a multiple of the period, and the
    owners send worker w their shards (and P's when a special update
    happened since w's last pull); w then computes its next gradient."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "distributed-deep-q_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ddq import dist as ddist
    from oracle import ref_numpy as ref
    ddist.init_process_group(rank, world, "gloo")
    P = 1000
    L = _shard_len(P, world)
    theta0 = np.random.default_rng(7).normal(0, 1, world * L).astype(np.float32)
    theta0[P:] = 0
    mine = slice(rank * L, (rank + 1) * L)
    own, pown, cache = theta0.copy(), theta0.copy(), None     # owner copies (own shard used)
    view, pview = theta0.copy(), theta0.copy()                # this worker's pulled model
    k = 0
    grad = _fake_grad(view[:P], rank, k)
    gfull = np.zeros(world * L, np.float32)
    it = 0
    for _ in range(rounds):
        for w in range(world):
            last = it + 1 - world if it + 1 - world > 0 else 0
            it += 1
            pull_p = it // period > last // period
            # push
            if rank == w:
                gfull[:P] = grad
                for j in range(world):
                    if j != rank:
                        dist.send(torch.from_numpy(gfull[j * L:(j + 1) * L].copy()), dst=j)
                sl = gfull[mine].copy()
            else:
                t = torch.zeros(L)
                dist.recv(t, src=w)
                sl = t.numpy()
            # owner apply on arrival
            shard, cache = ref.rmsprop_update(own[mine], sl, cache, 1e-2)
            own[mine] = shard
            cache = np.asarray(cache, np.float32)
            if it % period == 0:
                pown[mine] = own[mine]
            # pull
            if rank != w:
                dist.send(torch.from_numpy(own[mine].copy()), dst=w)
                if pull_p:
                    dist.send(torch.from_numpy(pown[mine].copy()), dst=w)
            else:
                for j in range(world):
                    src = slice(j * L, (j + 1) * L)
                    if j == rank:
                        view[src] = own[src]
                        if pull_p:
                            pview[src] = pown[src]
                        continue
                    t = torch.zeros(L)
                    dist.recv(t, src=j)
                    view[src] = t.numpy()
                    if pull_p:
                        t = torch.zeros(L)
                        dist.recv(t, src=j)
                        pview[src] = t.numpy()
                k += 1
                grad = _fake_grad(view[:P], rank, k)
    out.put((rank, view[:P].copy(), pview[:P].copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_async_round_robin_matches_server_replay(world):
    """Every worker's pulled model and P tower after 3 rounds equal the
    reference param server (server.py:181-209) serving W free-running workers
    whose pushes arrive round-robin: each gradient computed on the model its
    worker pulled one round earlier, applied on arrival; every pull at an
    iteration multiple of the special-update period copies Q to P first."""
    from oracle import ref_numpy as ref
    rounds, period = 3, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, rounds, period, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # sequential replay of the central server
    P = 1000
    L = _shard_len(P, world)
    theta0 = np.random.default_rng(7).normal(0, 1, world * L).astype(np.float32)[:P]
    central, pc, cache, it = theta0.copy(), theta0.copy(), None, 0
    view = [theta0.copy() for _ in range(world)]
    pview = [theta0.copy() for _ in range(world)]
    kk = [0] * world
    grads = [_fake_grad(theta0, w, 0) for w in range(world)]
    for _ in range(rounds):
        for w in range(world):
            central, cache = ref.rmsprop_update(central, grads[w], cache, 1e-2)
            cache = np.asarray(cache, np.float32)
            it += 1
            if it % period == 0:           # the pull sees iteration % period == 0
                pc = central.copy()
            view[w], pview[w] = central.copy(), pc.copy()
            kk[w] += 1
            grads[w] = _fake_grad(view[w], w, kk[w])
    for r, v, pv in res:
        np.testing.assert_allclose(v, view[r], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(pv, pview[r], rtol=1e-6, atol=1e-7)
    # staleness: the workers' views differ (each pulled at a different tick)
    assert not np.array_equal(res[0][1], res[1][1])


class _FakeAsyncNet:
    """The ddq_async_* surface of a worker whose gradient takes `compute_s`:
    it is ready that long after its last pull (its own tick)."""

    def __init__(self, rank, compute_s):
        import time
        self.rank, self.compute_s, self.time = rank, compute_s, time
        self.ticks = []
        self.pulled = None

    def async_begin(self, cfg):
        if self.pulled is None:
            self.pulled = self.time.perf_counter()

    def async_ready(self):
        return self.time.perf_counter() - self.pulled >= self.compute_s

    def async_tick(self, cfg, w):
        self.ticks.append(w)
        if w == self.rank:
            self.pulled = self.time.perf_counter()


def _ticket_worker(rank, world, port, npush, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "distributed-deep-q_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from ddq import dist as ddist
    ddist.init_process_group(rank, world, "gloo")
    net = _FakeAsyncNet(rank, 0.002 if rank == 0 else 0.012)
    loop = ddist.AsyncTicketLoop(net, None, ddist.ticket_store(world, rank), rank, world)
    order = loop.run(npush // 2) + loop.run(npush - npush // 2)   # two calls: state carries
    # a second loop on the same store keys its own tickets (no replay of the
    # first loop's): its ticket counter starts at 0
    loop2 = ddist.AsyncTicketLoop(net, None, ddist.ticket_store(world, rank), rank, world)
    order2 = loop2.run(6)
    taken2 = int(loop2.store.add("ticket", 0))
    out.put((rank, order, net.ticks[:npush], (loop2.instance, order2, taken2)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_async_ticket_order(world):
    """AsyncTicketLoop (the arrival-order async exchange's host side): every
    rank executes the same tick sequence, each ticket owned by the rank that
    took it when its gradient was ready, so the fast rank 0 pushes more often
    than the slow ones -- server.py applying pushes as they arrive."""
    npush = 30
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ticket_worker, args=(r, world, port, npush, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    orders = [r[1] for r in res]
    assert all(o == orders[0] for o in orders)
    assert all(r[2] == orders[0] for r in res)        # the ticks each rank enqueued
    assert len(orders[0]) == npush
    counts = np.bincount(orders[0], minlength=world)
    assert counts[0] > max(counts[1:]) and min(counts) >= 1, counts
    second = [r[3] for r in res]
    assert all(inst == 1 for inst, _, _ in second)
    assert all(o2 == second[0][1] and len(o2) == 6 for _, o2, _ in second)
    assert all(6 <= taken <= 6 + world for _, _, taken in second), second
