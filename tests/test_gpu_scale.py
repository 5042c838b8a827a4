"""GPU: the C4 / C5 worker counts (BASELINE.json configs 4 and 5) in-process.

The reference runs one Barista per partition, each with its own 30 000-slot
replay shard (ddq.py:40-70), all pushing to one parameter server
(server.py:196-209).  Here W = 8 contexts on one MI355X run the same kernels,
shard layout and exchange arithmetic as 8 RCCL ranks (ddq_group_step: the
collectives become device copies), at the headline shape (64x64, B = 32,
bench initialisation: seed-42 Gaussian fillers, zero biases):

* C4: 8 members x 30 000 slots, every exchange (allreduce, sharded, server),
  two rmsprop steps; every member's blobs and gradient against the oracle
  (rtol 1e-4 + 1e-6 * |terms|, tests/_parity.py), the members' parameters
  bit-identical, and the update against server.py's rules applied to the
  GPU's own gradients (in rank order for the server exchange).
* C5: 8 members x 1M-slot 64x64 rings (8 x 16.4 GB in HBM), the server
  exchange over two steps as above, then a 4096-transition device draw +
  gather per member checked row by row against its tiled pool.
* C5 as BASELINE.json states it -- 8 ASYNC workers with 1M-slot rings: two
  round-robin rounds (16 pushes, special update every 10 iterations) checked
  tick by tick against server.py replayed in the same arrival order
  (tests/_async_check.py), then a ticket-order run (ddq_group_async_run).
"""
import numpy as np
import pytest

from _parity import check_full_pass, close

pytestmark = pytest.mark.gpu

W, S, B = 8, 64, 32


@pytest.fixture(scope="module")
def ddq():
    import ddq as m
    return m


@pytest.fixture(scope="module")
def ref():
    from oracle import ref_numpy
    return ref_numpy


def apply_ref(ref, rule, theta, g, state, lr):
    if rule == "sgd":
        return ref.sgd_update(theta, g, lr), None
    if rule == "rmsprop":
        return ref.rmsprop_update(theta, g, state, lr)
    return ref.adagrad_update(theta, g, state, lr)


def pools(S, pool, seed):
    from ddq.expgain import synthetic_transitions
    st, ac, rw, nt = synthetic_transitions(pool, S, seed=seed)
    return st, ac, rw, nt.astype(np.uint8)


def make_members(ddq, N, pool, log=0):
    from ddq.params import init_params_flat
    theta = init_params_flat(S, seed=42)
    nets, data = [], []
    for r in range(W):
        n = ddq.DeepQNet(batch=B, frame=S)
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        d = pools(S, pool, seed=500 + r)          # each member its own shard contents
        n.replay_fill_tiled(*d, 0, N)
        if log:
            n.index_log_enable(log)
        nets.append(n)
        data.append(d)
    return nets, data, theta


def run_exchange(ddq, ref, nets, theta, exchange, rule="rmsprop", lr=1e-4, steps=2):
    grp = ddq.DeepQNet.group_init(nets)
    state = None
    for step in range(steps):
        cfg = nets[0].step_cfg(rule, lr=lr, target_period=10, exchange=exchange, seed=70 + step)
        ddq.DeepQNet.group_step(nets, cfg, grp)
        pq = ref.unflatten(theta, S, "Q")
        own, mags = [], []
        for r, n in enumerate(nets):
            mb = n.read_minibatch()
            pp = ref.unflatten(n.get_flat(1), S, "P")
            if exchange == "allreduce":
                # the grad buffer holds the sum: check blobs here, the sum below
                _, grads, _ = _blobs_only(ref, n, pq, pp, mb, "r%d " % r)
                own.append(ref.flatten(grads))
                routes = {i: n.pool_mask(i) for i in (1, 2, 3)}
                _, mg = ref.magnitudes(pq, pp, *mb, routes=routes)
                mags.append(ref.flatten(mg))
            else:
                check_full_pass(ref, n, pq, pp, mb, quiet=True, what="%s r%d " % (exchange, r))
        th = [n.get_flat(0) for n in nets]
        for t in th[1:]:
            np.testing.assert_array_equal(t, th[0])
        gpu_g = [n.get_grads_flat() for n in nets]
        if exchange == "allreduce":
            gsum = np.sum(np.stack(own).astype(np.float64), axis=0)
            msum = np.sum(np.stack(mags).astype(np.float64), axis=0)
            for g in gpu_g:
                close(g, gsum, mag=msum, what="allreduce sum", quiet=True)
            want, state = apply_ref(ref, rule, theta, gpu_g[0], state, lr)
        elif exchange == "sharded":
            gs = np.sum(np.stack(gpu_g).astype(np.float64), axis=0).astype(np.float32)
            want, state = apply_ref(ref, rule, theta, gs, state, lr)
        else:                                       # applied on arrival, rank order
            want = theta.copy()
            for g in gpu_g:
                want, state = apply_ref(ref, rule, want, g, state, lr)
        close(th[0], want, what="%s theta step %d" % (exchange, step))
        if state is not None:
            state = np.asarray(state, np.float32)
            close(owner_state(nets, exchange), state,
                  what="%s opt state step %d" % (exchange, step))
        theta = th[0]
    return theta


def owner_state(nets, exchange):
    """The optimizer state as the W owners hold it: allreduce keeps a full
    replica per member; sharded / server exchanges keep rank r's state only on
    its shard [r * L, (r + 1) * L), L = ceil(P / (64 W)) * 64 (api.hip
    setup_shards)."""
    if exchange == "allreduce":
        return nets[0].optimizer_state()
    P = nets[0].num_params
    L = -(-P // (64 * len(nets))) * 64
    out = np.empty(P, np.float32)
    for r, n in enumerate(nets):
        out[r * L:(r + 1) * L] = n.optimizer_state()[r * L:(r + 1) * L]
    return out


def _blobs_only(ref, net, pq, pp, mb, what):
    from _parity import full_pass_gpu_routing
    blobs, grads, nties = full_pass_gpu_routing(ref, net, pq, pp, mb)
    routes = {i: net.pool_mask(i) for i in (1, 2, 3)}
    mblobs, _ = ref.magnitudes(pq, pp, *mb, routes=routes)
    for name, shape in (("Q_out", (B, 4)), ("P_out", (B, 4)), ("Q_sa", (B,)), ("P_sa", (B,)),
                        ("target_Q_sa", (B,))):
        close(net.blob(name).reshape(shape), blobs[name], what=what + name, mag=mblobs[name],
              quiet=True)
    return blobs, grads, nties


@pytest.mark.parametrize("exchange", ["allreduce", "sharded", "server"])
def test_c4_eight_members_30k_shards(ddq, ref, exchange):
    nets, _, theta = make_members(ddq, 30000, pool=1024)
    try:
        run_exchange(ddq, ref, nets, theta, exchange)
    finally:
        for n in nets:
            n.close()


def test_c5_eight_members_million_slot_rings(ddq, ref):
    import torch
    N, pool, n = 1 << 20, 1024, 4096
    nets, data, theta = make_members(ddq, N, pool=pool)
    try:
        run_exchange(ddq, ref, nets, theta, "server")
        for r, (net, (st, ac, rw, nt)) in enumerate(zip(nets, data)):
            bufs = net.batch_buffers(n)
            net.replay_sample_batch(bufs, seed=900 + r)
            dev = bufs["idx"].device
            idx = bufs["idx"].long()
            assert bool((idx[1:] > idx[:-1]).all()) and int(idx[0]) >= 0 and int(idx[-1]) < N
            assert not bool((idx == N - 1).any())          # head 0: slot N-1 has no successor
            nxt = torch.where(idx + 1 == N, torch.zeros_like(idx), idx + 1)
            pst = torch.from_numpy(st).to(dev)
            assert torch.equal(bufs["state"], pst[idx % pool].float())
            assert torch.equal(bufs["next_state"], pst[nxt % pool].float())
            pac = torch.from_numpy(ac.astype(np.int64)).to(dev)[nxt % pool]
            assert torch.equal(bufs["action"].view(n, 4).argmax(1), pac)
            assert torch.equal(bufs["reward"].view(n),
                               torch.from_numpy(rw.astype(np.float32)).to(dev)[nxt % pool])
            assert torch.equal(bufs["non_terminal"].view(n),
                               torch.from_numpy(nt.astype(np.float32)).to(dev)[nxt % pool])
            del bufs
    finally:
        for net in nets:
            net.close()


def test_c5_eight_async_workers_million_slot_rings(ddq, ref):
    from _async_check import run_checked
    N, pool = 1 << 20, 1024
    nets, data, theta = make_members(ddq, N, pool=pool, log=64)
    try:
        arr = ddq.DeepQNet.group_init(nets)

        def minibatch(r, draw):        # member r's draw: its tiled pool at the logged indices
            st, ac, rw, nt = data[r]
            idx = nets[r].index_log(draw, 1)[0].astype(np.int64)
            nx = np.where(idx + 1 == N, 0, idx + 1)
            a = np.zeros((B, 4, 1, 1), np.float32)
            a[np.arange(B), ac[nx % pool], 0, 0] = 1
            return (st[idx % pool].astype(np.float32), a,
                    rw[nx % pool].astype(np.float32).reshape(B, 1, 1, 1),
                    st[nx % pool].astype(np.float32),
                    nt[nx % pool].astype(np.float32).reshape(B, 1, 1, 1))
        lr, period = 1e-4, 10
        cfg = nets[0].step_cfg("rmsprop", lr=lr, target_period=period, exchange="async", seed=77)
        order = list(range(W)) * 2                 # two round-robin rounds
        # every gradient is checked at the first pushes; later ones 1 in 3
        run_checked(ddq, ref, nets, arr, cfg, order, minibatch, "rmsprop", lr, period, theta,
                    grad_check=lambda t, w: (t < 0 and w < 2) or (t >= 0 and t % 3 == 0),
                    what="C5 ")
        # arrival order: 24 more pushes by whichever worker is ready first
        before = [n.get_flat(0) for n in nets]
        got = ddq.DeepQNet.group_async_run(nets, cfg, 24, arr)
        assert len(got) == 24 and set(got.tolist()) <= set(range(W))
        for n, b in zip(nets, before):
            th = n.get_flat(0)
            assert np.isfinite(th).all()
        assert any(not np.array_equal(n.get_flat(0), b) for n, b in zip(nets, before))
    finally:
        for n in nets:
            n.close()
