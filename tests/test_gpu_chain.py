"""A20 end to end: the SHIPPED step path against the oracle.

The bench default is ``ddq_step_pipelined_async`` at BASELINE configs[1]
(64x64, B=32): 8-step hipGraphs plus tail graphs, the next step's device draw
+ gather carried by the slab-reduce launch, the fc4-weight update fused into
that launch, the rest of the apply in its own launch, P <- Q fused into the
apply before every pull that sees iteration % 10 == 0.  Chains of that path
run from the bench's own initial state (seed-42 Gaussian fillers, zero biases,
P = Q, a 30 000-slot ring of synthetic random-policy Snake frames) with the
device index log on, and the oracle replays the reference's worker/server
loop on exactly the logged minibatches:

  pull: if iteration % 10 == 0: P <- Q      (param-server/server.py:181-193)
  gather(idx)                                (replay.py:159-183)
  full_pass                                  (baristanet.py:138-140)
  apply_descent with the rule                (server.py:49-124; rmsprop's
                                              lagged cache :86-105)

Why two tests.  The reference's rmsprop divides by the PREVIOUS step's cache
(lr*g/sqrt(g_prev^2 + 1e-8)): wherever g_prev ~ 0 the update is ~g itself, a
10^4-fold amplification of lr, so two fp32/fp64 trajectories separate once a
single near-tie (a max-pool window or ReLU input within fp32 rounding of its
alternative) resolves differently -- measured on this workload: the free-
running gradient error jumps from ~4e-9 to ~1e-5 at step 7 and grows to the
size of the gradient by step ~15 (tools/gpu/dbg_chain.py).  Any fp32
implementation, Caffe's CPU path included, shows the same against a float64
oracle.  So:

* ``test_shipped_chain_teacher_forced`` (31 steps, rmsprop and sgd): the
  shipped pipelined chain (calls of 25 + 6 steps: three 8-step graphs, a
  single-step graph, a 6-step tail graph; P <- Q at 10, 20, 30) is BIT-
  IDENTICAL to the sequence of eager ``ddq_step_async`` steps, and every one
  of those 31 steps, started from the GPU's own state, matches the oracle's
  step (gradients, theta_Q, theta_P, optimizer state, loss) at rtol 1e-4
  with the GPU's max-pool routing adopted only at proven near-ties.
* ``test_shipped_chain_free_running``: the chain from the common initial
  state against a free-running oracle, rtol 1e-4 on theta_Q, theta_P, the
  cache and the loss: 6 rmsprop steps (its lagged cache divides by earlier
  gradients, amplifying fp32-vs-fp64 differences of near-zero elements) and
  24 sgd steps (two P <- Q syncs).
"""
import numpy as np
import pytest

from _parity import close

pytestmark = pytest.mark.gpu

S, B, N = 64, 32, 30000


@pytest.fixture(scope="module")
def ref_mod():
    from oracle import ref_numpy
    return ref_numpy


_RINGS = {}


def ring_for(S):
    """The bench's replay contents at 64x64 (bench.fill_replay, rank 0: a 4096-
    transition pool tiled over 30 000 slots); at 16x16 (deepq16) 4096 slots."""
    if S not in _RINGS:
        from ddq.expgain import synthetic_transitions
        pool = 4096
        n = N if S == 64 else pool
        st, ac, rw, nt = synthetic_transitions(pool, S, seed=1000 if S == 64 else 77)
        reps = (n + pool - 1) // pool
        _RINGS[S] = (np.tile(st, (reps, 1, 1, 1))[:n], np.tile(ac, reps)[:n],
                     np.tile(rw, reps)[:n], np.tile(nt, reps)[:n])
    return _RINGS[S]


@pytest.fixture(scope="module")
def ring():
    return ring_for(S)


def oracle_chain(ref, theta, ring_arrays, log, rule, lr, period, S=S):
    st, ac, rw, nt = ring_arrays
    N = len(st)
    r = ref.ReplayRef((4, S, S), N)
    r.state, r.action, r.reward, r.non_terminal = st, ac, rw, nt.astype(bool)
    r.head, r.valid = 0, N
    thq = theta.astype(np.float32).copy()
    thp = thq.copy()
    state = None
    loss = None
    for t, idx in enumerate(log):
        if period and t % period == 0:           # the pull at iteration t
            thp = thq.copy()
        mb = r.gather(idx)
        blobs, grads = ref.full_pass(ref.unflatten(thq, S, "Q"), ref.unflatten(thp, S, "P"),
                                     *mb)
        loss = blobs["loss"]
        g = ref.flatten(grads).astype(np.float32)   # the fp32 gradient message
        if rule == "rmsprop":
            thq, state = ref.rmsprop_update(thq, g, state, lr, 0.9)
        elif rule == "sgd":
            thq = ref.sgd_update(thq, g, lr)
        else:
            raise ValueError(rule)
    if period and len(log) % period == 0:        # the sync fused into the last apply
        thp = thq.copy()
    return thq, thp, state, loss


def make_net(ddq, theta, ring, log=64, S=S, B=B):
    N = len(ring[0])
    net = ddq.DeepQNet(batch=B, frame=S)
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    net.replay_create(N)
    st, ac, rw, nt = ring
    net.replay_import(st, ac, rw, nt.astype(np.uint8), 0, N)
    net.index_log_enable(log)
    return net


def oracle_rule(ref, rule, th, g, state, lr):
    if rule == "rmsprop":
        return ref.rmsprop_update(th, g, state, lr, 0.9)
    if rule == "sgd":
        return ref.sgd_update(th, g, lr), None
    raise ValueError(rule)


# (S, B, rule, lr, calls): the bench's C2 step (64x64) and deepq16 (16x16,
# train_val.prototxt:8-11: the four-launch small-map step the bench's deepq16
# line measures, with its fused apply in K2 / K4), plus deepq16 at C3's B = 256
# (the fc4 chain in 8 image chunks, their partial sums applied by K4)
TEACHER_FORCED = [(64, 32, "rmsprop", 1e-4, (25, 6)), (64, 32, "sgd", 1e-2, (17, 3, 1, 10)),
                  (16, 32, "rmsprop", 1e-4, (25, 6)), (16, 32, "sgd", 1e-2, (17, 3, 1, 10)),
                  (16, 256, "rmsprop", 1e-4, (9, 3))]


@pytest.mark.parametrize("S,B,rule,lr,calls", TEACHER_FORCED)
def test_shipped_chain_teacher_forced(ref_mod, S, B, rule, lr, calls):
    import ddq
    from ddq.params import init_params_flat
    from _parity import check_full_pass
    ref = ref_mod
    ring = ring_for(S)
    N = len(ring[0])
    theta = init_params_flat(S, seed=42)
    T = sum(calls)
    chain = make_net(ddq, theta, ring, S=S, B=B)
    if S == 16:
        assert chain.small_path()[0], chain.small_path()
    cfg = chain.step_cfg(rule, lr=lr, target_period=10, seed=1234)
    for k in calls:
        chain.step_pipelined(cfg, k)
    chain.synchronize()
    chain._check(chain.lib.ddq_replay_status(chain.ctx))
    assert chain.replay_draws() == T
    log = chain.index_log(0, T)
    for idx in log:
        assert np.all(np.diff(idx) > 0) and idx[0] >= 0 and idx[-1] < N
    np.testing.assert_array_equal(chain.read_indices(), log[-1])

    st, ac, rw, nt = ring
    r = ref.ReplayRef((4, S, S), N)
    r.state, r.action, r.reward, r.non_terminal = st, ac, rw, nt.astype(bool)
    r.head, r.valid = 0, N
    eager = make_net(ddq, theta, ring, S=S, B=B)
    thq, thp = theta.copy(), theta.copy()
    state = None
    ties = 0
    for t in range(T):
        eager.step(cfg)
        eager.synchronize()
        idx = eager.read_indices()
        np.testing.assert_array_equal(idx, log[t])           # same draw as the chain
        # the oracle's step from the GPU's own state before it
        p_pull = thq if t % 10 == 0 else thp                  # the pull's P <- Q
        mb = r.gather(idx)
        blobs, grads, n = check_full_pass(ref, eager, ref.unflatten(thq, S, "Q"),
                                          ref.unflatten(p_pull, S, "P"), mb,
                                          what="step %d " % t, quiet=t not in (0, T - 1))
        ties += n
        g = ref.flatten(grads).astype(np.float32)
        th_ref, st_ref = oracle_rule(ref, rule, thq, g, state, lr)
        gq, gp = eager.get_flat(0), eager.get_flat(1)
        close(gq, th_ref, what="step %d theta_Q" % t, quiet=t not in (0, T - 1))
        np.testing.assert_array_equal(gp, gq if (t + 1) % 10 == 0 else p_pull)
        if rule != "sgd":
            gst = eager.optimizer_state()
            close(gst, st_ref, what="step %d cache" % t, quiet=t not in (0, T - 1))
            state = gst
        thq, thp = gq, gp
    print("%dx%d B=%d %s: %d teacher-forced steps at rtol 1e-4, %d near-tie routings adopted"
          % (S, S, B, rule, T, ties))
    # the shipped chain IS that sequence of steps, bit for bit
    np.testing.assert_array_equal(chain.get_flat(0), eager.get_flat(0))
    np.testing.assert_array_equal(chain.get_flat(1), eager.get_flat(1))
    np.testing.assert_array_equal(chain.optimizer_state(), eager.optimizer_state())
    np.testing.assert_array_equal(chain.index_log(0, T), eager.index_log(0, T))
    assert float(chain.blob("loss")) == float(eager.blob("loss"))
    chain.close()
    eager.close()


@pytest.mark.parametrize("rule,lr,calls", [("rmsprop", 1e-4, (1, 5)), ("sgd", 1e-2, (16, 8))])
def test_shipped_chain_free_running(ref_mod, ring, rule, lr, calls):
    import ddq
    from ddq.params import init_params_flat
    ref = ref_mod
    theta = init_params_flat(S, seed=42)
    net = make_net(ddq, theta, ring)
    T = sum(calls)
    cfg = net.step_cfg(rule, lr=lr, target_period=10, seed=1234)
    for k in calls:
        net.step_pipelined(cfg, k)
    net.synchronize()
    log = net.index_log(0, T)
    thq, thp, state, loss = oracle_chain(ref, theta, ring, log, rule, lr, 10)
    gq, gp = net.get_flat(0), net.get_flat(1)
    assert not np.array_equal(gq, theta)
    close(gq, thq, what="%s theta_Q after %d" % (rule, T))
    close(gp, thp, what="%s theta_P after %d" % (rule, T))
    if state is not None:
        close(net.optimizer_state(), state, what="%s cache after %d" % (rule, T))
    close(float(net.blob("loss")), loss, what="%s loss of step %d" % (rule, T))


def test_deepq16_chain_free_running_48_sgd(ref_mod):
    """48 free-running sgd steps of the shipped pipelined chain at the
    reference's committed shape (deepq16: 16x16, B = 32; train_val.prototxt
    :8-11), four P <- Q syncs, against the oracle replaying the reference's
    loop on the logged minibatches: theta_Q, theta_P and the loss at rtol 1e-4
    after the whole chain (calls of 20 + 5 + 23 steps: 8-step graphs, tail
    graphs, single steps)."""
    import ddq
    from ddq.expgain import synthetic_transitions
    from ddq.params import init_params_flat
    S16, N16 = 16, 4096
    ring16 = synthetic_transitions(N16, S16, seed=77)
    theta = init_params_flat(S16, seed=42)
    net = make_net(ddq, theta, ring16, log=64, S=S16)
    calls = (20, 5, 23)
    T = sum(calls)
    cfg = net.step_cfg("sgd", lr=1e-2, target_period=10, seed=4321)
    for k in calls:
        net.step_pipelined(cfg, k)
    net.synchronize()
    log = net.index_log(0, T)
    thq, thp, _, loss = oracle_chain(ref_mod, theta, ring16, log, "sgd", 1e-2, 10, S=S16)
    gq, gp = net.get_flat(0), net.get_flat(1)
    assert not np.array_equal(gq, theta)
    close(gq, thq, what="sgd theta_Q after %d" % T)
    close(gp, thp, what="sgd theta_P after %d" % T)
    close(float(net.blob("loss")), loss, what="sgd loss of step %d" % T)
    net.close()
