"""GPU: data-parallel gradient exchanges (include/ddq_hip.h enum
ddq_exchange) against the param-server semantics of server.py:196-209.

* In-process groups (ddq_group_init / ddq_group_step): W ctxs on one GPU run
  the same kernels, shard layout and exchange arithmetic as RCCL ranks, with
  the collectives done as device copies -- the sharded and server exchanges
  are checked here against the oracle's update rules:
    server    : theta' = apply(...apply(apply(theta, g_0), g_1)..., g_{W-1})
                (each gradient applied on arrival, in rank order; rmsprop's
                lagged cache and first call carried across them; iteration
                += W per step, so the P <- Q pull check sees W-multiples);
    sharded / allreduce : theta' = apply(theta, sum_r g_r).
* RCCL with a 1-rank communicator: every exchange (incl. the overlapped
  all-reduce inside the step graph) equals the exchange-free step bit-exactly.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def close(a, b, scale, rtol=1e-5, what=""):
    err = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    tol = rtol * (np.abs(b) + scale)
    assert (err <= tol).all(), "%s: max err %.3g" % (what, err.max())


def make_group(ddq, ref, W, S=16, B=8, N=120, seed=0):
    theta = ref.flatten(ref.init_params(S, seed=21))
    theta = (theta * 3).astype(np.float32)
    nets = []
    for r in range(W):
        rng = np.random.default_rng(seed + r)
        n = ddq.DeepQNet(batch=B, frame=S)
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8),
                        rng.integers(0, 4, N).astype(np.uint8),
                        rng.integers(-1, 2, N).astype(np.int16),
                        (rng.random(N) > 0.1).astype(np.uint8), 0, N)
        nets.append(n)
    arr = ddq.DeepQNet.group_init(nets)
    return nets, arr, theta


@pytest.mark.parametrize("exchange", ["server", "sharded", "allreduce"])
@pytest.mark.parametrize("rule", ["rmsprop", "adagrad", "sgd"])
def test_group_exchange_semantics(ddq, ref, exchange, rule):
    # Two steps: the second runs on the first's optimizer state.  (The lagged
    # rmsprop cache of server.py:86-105 lets a later gradient divide by an
    # earlier, tiny one -- steps of up to lr*|g|*1e4 -- so longer runs at
    # these raw-pixel gradient scales leave the finite range, in the
    # reference as here.)
    W, S, lr = 3, 16, 1e-4
    nets, arr, theta = make_group(ddq, ref, W, S)
    state = None
    for step in range(2):
        cfg = nets[0].step_cfg(rule, lr=lr, target_period=0, exchange=exchange, seed=40 + step)
        # one cfg (seed) for the group: the members' minibatches differ
        # through their own replay contents
        ddq.DeepQNet.group_step(nets, cfg, arr)
        # per-rank gradients at the common theta, from each rank's own minibatch
        grads = []
        for n in nets:
            st, ac, rw, ns, nt = n.read_minibatch()
            pq, pp = ref.unflatten(theta, S, "Q"), ref.unflatten(n.get_flat(1) if step else theta,
                                                               S, "P")
            _, g = ref.full_pass(pq, pp, st, ac, rw, ns, nt)
            grads.append(ref.flatten(g).astype(np.float32))
        if exchange != "allreduce":           # own gradient stays in the grad buffer
            for n, g in zip(nets, grads):
                close(n.get_grads_flat(), g, np.abs(g).max(), 1e-4, "grad")
        else:                                 # the buffer holds the sum on every rank
            gsum = np.sum(np.stack(grads).astype(np.float64), axis=0)
            for n in nets:
                close(n.get_grads_flat(), gsum, np.abs(gsum).max(), 1e-4, "grad sum")
        # the members agree bit-exactly
        th = [n.get_flat(0) for n in nets]
        for t in th[1:]:
            np.testing.assert_array_equal(t, th[0])
        # oracle apply with the GPU's own gradients where they are observable
        gpu_g = [n.get_grads_flat() for n in nets]
        if exchange == "server":
            want = theta.copy()
            for g in gpu_g:
                want, state = apply_ref(ref, rule, want, g, state, lr)
        elif exchange == "sharded":
            gs = np.sum(np.stack(gpu_g).astype(np.float64), axis=0).astype(np.float32)
            want, state = apply_ref(ref, rule, theta, gs, state, lr)
        else:
            want, state = apply_ref(ref, rule, theta, gpu_g[0], state, lr)
        close(th[0], want, np.abs(theta - want).max() + 1e-30, 1e-3, "theta step %d" % step)
        theta = th[0]
        if state is not None:
            state = np.asarray(state, np.float32)
    for n in nets:
        n.close()


def test_group_server_iteration_and_target_sync(ddq, ref):
    """server mode counts W iterations per step; P <- Q when the pull after
    a step sees iteration % period == 0 (server.py:188-189)."""
    W, S = 3, 16
    nets, arr, theta = make_group(ddq, ref, W, S)
    cfg = nets[0].step_cfg("sgd", lr=1e-2, target_period=2, exchange="server", seed=3)
    ddq.DeepQNet.group_step(nets, cfg, arr)      # iteration 3: no sync
    for n in nets:
        assert not np.array_equal(n.get_flat(1), n.get_flat(0))
        np.testing.assert_array_equal(n.get_flat(1), theta)
    ddq.DeepQNet.group_step(nets, cfg, arr)      # iteration 6: sync
    for n in nets:
        np.testing.assert_array_equal(n.get_flat(1), n.get_flat(0))
    for n in nets:
        n.close()


@pytest.mark.parametrize("exchange,overlap", [("allreduce", False), ("allreduce", True),
                                              ("sharded", False), ("server", False)])
def test_rccl_world1_exchange_equals_plain_step(ddq, ref, exchange, overlap):
    S, B, N = 16, 8, 96
    rng = np.random.default_rng(4)
    theta = (ref.flatten(ref.init_params(S, seed=5)) * 3).astype(np.float32)
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    ac = rng.integers(0, 4, N).astype(np.uint8)
    rw = rng.integers(-1, 2, N).astype(np.int16)
    nt = (rng.random(N) > 0.1).astype(np.uint8)
    nets = [ddq.DeepQNet(batch=B, frame=S) for _ in range(2)]
    for n in nets:
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(st, ac, rw, nt, 0, N)
    nets[0].comm_init(ddq.DeepQNet.comm_unique_id(), 1, 0)
    for i, n in enumerate(nets):
        cfg = n.step_cfg("rmsprop", lr=1e-3, target_period=3,
                         exchange=exchange if i == 0 else "none", overlap=overlap, seed=9)
        n.step_graph(cfg, 5)
        n.step(cfg)
        n.synchronize()
    for z in (0, 1):
        np.testing.assert_array_equal(nets[0].get_flat(z), nets[1].get_flat(z))
    np.testing.assert_array_equal(nets[0].optimizer_state(), nets[1].optimizer_state())
    for n in nets:
        n.close()
