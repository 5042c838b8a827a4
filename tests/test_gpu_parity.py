"""GPU parity: libddq_hip.so (through the C-ABI) vs the oracle.

Tolerances (north star: "Q-values, targets, gradients and post-update weights
must match within fp32 rtol 1e-4"):
  * integer / index / byte work (replay gather, argmax actions): bit-exact;
  * fp32 tensors: tests/_parity.py ``close`` -- elementwise rtol 1e-4 for every
    element with |ref| >= 1e-3 of the tensor's scale, the same rtol on that
    1e-3 floor below it; the oracle runs in float64.
"""
import glob
import os

import numpy as np
import pytest

from _parity import check_full_pass, close

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def ddq():
    import ddq as m
    return m


@pytest.fixture(scope="module")
def ref():
    from oracle import ref_numpy
    return ref_numpy


# ---------------------------------------------------------------- replay (A1-A3)
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(
    os.path.dirname(__file__), "golden", "replay_*.npz"))))
def test_replay_gather_bitexact_vs_reference(ddq, path):
    f = np.load(path)
    S, N, B = int(f["S"]), int(f["N"]), int(f["B"])
    net = ddq.DeepQNet(batch=B, frame=S)
    net.replay_create(N)
    net.replay_import(f["st"], f["action"], f["reward"], f["non_terminal"].astype(np.uint8),
                      int(f["head"]), int(f["valid"]))
    if str(f["error"]):
        with pytest.raises(ddq._lib.DDQError) as ei:
            net.replay_sample(np.arange(B, dtype=np.int32))
        assert "Can't draw sample of size %d from replay dataset of size %d" % (
            B, int(f["valid"])) in str(ei.value)
        return
    net.replay_sample(f["idx"])
    st, ac, rw, ns, nt = net.read_minibatch()
    np.testing.assert_array_equal(st, f["out_state"])
    np.testing.assert_array_equal(ns, f["out_next_state"])
    np.testing.assert_array_equal(ac, f["out_action"])
    np.testing.assert_array_equal(rw, f["out_reward"])
    np.testing.assert_array_equal(nt, f["out_non_terminal"])


def test_replay_add_matches_reference_ring(ddq, ref):
    """add_experience ring semantics incl. stale terminal slots and wrap."""
    S, N = 16, 8
    rng = np.random.default_rng(3)
    net = ddq.DeepQNet(batch=4, frame=S)
    net.replay_create(N)
    r = ref.ReplayRef((4, S, S), N)
    for i in range(21):
        st = None if i % 3 == 2 else rng.integers(0, 256, (4, S, S)).astype(np.uint8)
        a, rw = int(rng.integers(0, 4)), int(rng.integers(-1, 2))
        net.replay_add(a, rw, st)
        r.add_experience(a, rw, st)
    h, v, c = net.replay_info()
    assert (h, v, c) == (r.head, r.valid, N)
    st, ac, rw, nt = net.replay_export()
    np.testing.assert_array_equal(st, r.state)
    np.testing.assert_array_equal(ac, r.action)
    np.testing.assert_array_equal(rw, r.reward)
    np.testing.assert_array_equal(nt, r.non_terminal)


def test_device_sampler_properties(ddq):
    """Device index draw: sorted, distinct, in [0, valid), never head-1."""
    S, N, B = 16, 64, 32
    net = ddq.DeepQNet(batch=B, frame=S)
    net.replay_create(N)
    rng = np.random.default_rng(0)
    for i in range(N + 7):          # wrapped: head = 7, head-1 = 6 forbidden
        net.replay_add(i % 4, 0, rng.integers(0, 256, (4, S, S)).astype(np.uint8))
    head, valid, _ = net.replay_info()
    seen = np.zeros(valid, int)
    for it in range(200):
        net.replay_sample_device(seed=1234)
        idx = net.read_indices()
        assert np.all(np.diff(idx) > 0)
        assert idx.min() >= 0 and idx.max() < valid
        assert (head - 1) not in idx
        seen[idx] += 1
    assert seen[head - 1] == 0
    # roughly uniform over the other valid - 1 slots (32/63 each draw)
    others = np.delete(seen, head - 1)
    assert others.min() > 0.5 * 200 * B / (valid - 1)


@pytest.mark.parametrize("B", [32, 96])
def test_device_sampler_nearly_full_population(ddq, B):
    """valid = B + 1 (the smallest population replay.py:147-150 accepts): every
    draw must still be a distinct sorted set (redraws continue until it is;
    a set that cannot be completed is reported by ddq_replay_status, never
    gathered silently).  B = 96 takes the multi-wave (bitonic) sampler."""
    S, N = 16, B + 1
    net = ddq.DeepQNet(batch=B, frame=S)
    net.replay_create(N)
    rng = np.random.default_rng(4)
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    net.replay_import(st, np.zeros(N, np.uint8), np.zeros(N, np.int16), np.ones(N, np.uint8),
                      0, N)
    missing = set()
    for it in range(40):
        net.replay_sample_device(seed=99)
        net._check(net.lib.ddq_replay_status(net.ctx))
        idx = net.read_indices()
        assert np.all(np.diff(idx) > 0) and idx[0] >= 0 and idx[-1] < N
        missing |= set(range(N)) - set(idx.tolist())
    assert len(missing) > 1          # different sets across draws


# ------------------------------------------------------- full pass (A8-A13)
def make_inputs(rng, B, S, frames="uniform"):
    if frames == "uniform":
        st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
        ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    elif frames == "snake":   # snake-like sparse frames {0, 200, 255}
        st = rng.choice(np.array([0, 200, 255], np.float32), (B, 4, S, S), p=[0.9, 0.08, 0.02])
        ns = rng.choice(np.array([0, 200, 255], np.float32), (B, 4, S, S), p=[0.9, 0.08, 0.02])
    else:                     # the bench's frames: a replay.py gather of synthetic Snake play
        from ddq.expgain import synthetic_transitions
        from oracle import ref_numpy as ref
        n = max(4 * B, 512)
        sst, sac, srw, snt = synthetic_transitions(n, S, seed=int(rng.integers(1 << 30)))
        r = ref.ReplayRef((4, S, S), n)
        r.state, r.action, r.reward, r.non_terminal = sst, sac, srw, snt
        r.head, r.valid = 0, n
        st, act, rw, ns, nt = r.gather(np.sort(rng.choice(n - 1, B, replace=False)))
        return st, act, rw, ns, nt
    act = np.zeros((B, 4, 1, 1), np.float32)
    act[np.arange(B), rng.integers(0, 4, B)] = 1
    rw = rng.integers(-1, 2, (B, 1, 1, 1)).astype(np.float32)
    nt = (rng.random((B, 1, 1, 1)) > 0.2).astype(np.float32)
    return st, act, rw, ns, nt


def make_params(ref, rng, S, init):
    """init "x3": fillers x3 + random biases (activations O(1), no Q_out == 0);
    "bench": the bench's own seed-42 fillers, zero biases, P = Q."""
    if init == "bench":
        pQ = ref.init_params(S, seed=42, prefix="Q")
        pP = ref.init_params(S, seed=42, prefix="P")
        return pQ, pP
    pQ = ref.init_params(S, seed=7, prefix="Q")
    pP = ref.init_params(S, seed=8, prefix="P")
    for p in (pQ, pP):
        for k in p:
            p[k][0] = (p[k][0] * 3).astype(np.float32)
            p[k][1] = rng.normal(0, 0.05, p[k][1].shape).astype(np.float32)
    return pQ, pP


FULL_PASS_CASES = [
    (16, 32, "uniform", "x3"), (16, 32, "snake", "x3"), (24, 8, "uniform", "x3"),
    (40, 4, "snake", "x3"), (64, 32, "uniform", "x3"), (16, 256, "snake", "x3"),
    (128, 2, "uniform", "x3"), (72, 4, "snake", "x3"), (96, 4, "uniform", "x3"),
    # the bench's initial state on its own frames (C1 / C2 shapes)
    (16, 32, "bench", "bench"), (64, 32, "bench", "bench"),
    # C3: batch 256 across the frame sweep (results/cost-vs-image-size-trials.txt)
    (24, 256, "snake", "x3"), (64, 256, "bench", "bench"), (128, 256, "snake", "x3"),
    (104, 256, "snake", "x3"),
    # C3 B = 256 at the frames whose tiles leave partial edge tiles
    (40, 256, "snake", "x3"), (72, 256, "uniform", "x3"), (120, 256, "snake", "x3"),
    # the rest of the sweep's frames 16..128 / 8 (conv tilings incl. the
    # partial edge tiles of 40, 72, 104 and 120)
    (32, 4, "uniform", "x3"), (48, 4, "snake", "x3"), (56, 4, "uniform", "x3"),
    (80, 4, "snake", "x3"), (88, 4, "uniform", "x3"), (104, 4, "snake", "x3"),
    (112, 4, "uniform", "x3"), (120, 4, "snake", "x3"),
    # the small-map step's group splits: one group per tile (B = 1, 2), a
    # slice longer than one chunk (B = 8: two conv3 groups), ragged groups
    (16, 1, "snake", "x3"), (16, 2, "uniform", "x3"), (16, 8, "snake", "x3"),
    (16, 12, "uniform", "x3"), (16, 100, "snake", "x3"),
    # S = 16 past the small-map step's B <= 256: the general kernels
    (16, 300, "snake", "x3"),
]


@pytest.mark.parametrize("S,B,frames,init", FULL_PASS_CASES)
def test_full_pass_parity(ddq, ref, S, B, frames, init):
    rng = np.random.default_rng(100 + S + B)
    pQ, pP = make_params(ref, rng, S, init)
    net = ddq.DeepQNet(batch=B, frame=S)
    params = dict(pQ)
    params.update(pP)
    net.set_params(params)
    st, act, rw, ns, nt = make_inputs(rng, B, S, frames)
    net.write_minibatch(st, act, rw, ns, nt)
    loss = net.forward_backward()
    # Pool routing bit-exact except at proven fp32-vs-fp64 near-ties (GPU
    # routing adopted there); every blob and gradient element within
    # rtol 1e-4 + 1e-6 * (its sum of |terms|) (tests/_parity.py).
    blobs, _, nties = check_full_pass(ref, net, pQ, pP, (st, act, rw, ns, nt))
    assert loss == float(net.blob("loss"))
    print("near-tie routings adopted: %d" % nties)


@pytest.mark.parametrize("rule", ["sgd", "rmsprop", "adagrad", "momentum"])
def test_apply_rules_parity(ddq, ref, rule):
    S = 16
    rng = np.random.default_rng(11)
    net = ddq.DeepQNet(batch=8, frame=S)
    theta = ref.flatten(ref.init_params(S, seed=3))
    net.set_flat(0, theta)
    net.reset_optimizer()
    P = theta.size
    state = None
    th = theta.copy()
    # bias mask for the momentum rule multipliers (blobs_lr {1,2}, weight_decay {1,0})
    is_bias = np.zeros(P, bool)
    for qname, blobs in net.layout.items():
        s, o, c = blobs[1]
        is_bias[o:o + c] = True
    for step in range(3):
        g = (rng.normal(0, 1e-2, P)).astype(np.float32)
        net.set_grads_flat(g)
        net.apply(rule, lr=1e-3 if rule != "momentum" else 0.01)
        if rule == "sgd":
            th = ref.sgd_update(th, g, 1e-3)
        elif rule == "rmsprop":
            th, state = ref.rmsprop_update(th, g, state, 1e-3, 0.9)
        elif rule == "adagrad":
            th, state = ref.adagrad_update(th, g, state, 1e-3)
        else:
            v = np.zeros(P, np.float32) if state is None else state
            th, state = ref.momentum_caffe_update(th, g, v, np.where(is_bias, 2.0, 1.0).astype(np.float32),
                                                  np.where(is_bias, 0.0, 1.0).astype(np.float32))
        close(net.get_flat(0), th, what="%s step %d" % (rule, step))
        if state is not None:
            close(net.optimizer_state(), state, what="%s state %d" % (rule, step))


def test_target_sync_and_select_action(ddq, ref):
    S, B = 16, 8
    rng = np.random.default_rng(5)
    net = ddq.DeepQNet(batch=B, frame=S)
    pQ = ref.init_params(S, seed=21)
    for k in pQ:
        pQ[k][0] = (pQ[k][0] * 3).astype(np.float32)
        pQ[k][1] = rng.normal(0, 0.05, pQ[k][1].shape).astype(np.float32)
    net.set_params(pQ)
    net.sync_target()
    np.testing.assert_array_equal(net.get_flat(1), net.get_flat(0))
    states = rng.integers(0, 256, (5, 4, S, S)).astype(np.uint8)
    a = net.select_action(states)
    np.testing.assert_array_equal(a, ref.select_action(states.astype(np.float32), pQ))


def test_graph_step_runs_and_matches_eager(ddq, ref):
    """The fused device step (sample->gather->fwd/bwd->apply, hipGraph) equals the
    eager API sequence on the same indices."""
    S, B, N = 16, 16, 200
    rng = np.random.default_rng(9)
    nets = [ddq.DeepQNet(batch=B, frame=S) for _ in range(2)]
    theta = ref.flatten(ref.init_params(S, seed=4))
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    acts = rng.integers(0, 4, N).astype(np.uint8)
    rws = rng.integers(-1, 2, N).astype(np.int16)
    nts = (rng.random(N) > 0.1).astype(np.uint8)
    for n in nets:
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(st, acts, rws, nts, 0, N)
    cfg = nets[0].step_cfg("sgd", lr=1e-4, target_period=3, seed=77)
    nets[0].step_graph(cfg, 5)
    nets[0].synchronize()
    # eager replica: same device RNG stream through the async sampler
    e = nets[1]
    for t in range(5):
        if t % 3 == 0:
            e.sync_target()
        e.replay_sample_device(77)
        e.forward_backward()
        e.apply("sgd", lr=1e-4)
    th = nets[0].get_flat(0)
    assert np.all(np.isfinite(th))
    close(th, e.get_flat(0), rtol=1e-6, what="theta after 5 graph steps")
    np.testing.assert_array_equal(nets[0].read_indices(), e.read_indices())


def test_pipelined_step_matches_graph(ddq, ref):
    """Double-buffered pipelined stepping (next sample + gather under the
    current step) gives the same parameters, indices and minibatch as the
    plain graph step sequence, across several calls of different lengths."""
    S, B, N = 16, 16, 300
    rng = np.random.default_rng(21)
    nets = [ddq.DeepQNet(batch=B, frame=S) for _ in range(2)]
    theta = ref.flatten(ref.init_params(S, seed=6))
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    acts = rng.integers(0, 4, N).astype(np.uint8)
    rws = rng.integers(-1, 2, N).astype(np.int16)
    nts = (rng.random(N) > 0.1).astype(np.uint8)
    for n in nets:
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(st, acts, rws, nts, 0, N)
    cfg = nets[0].step_cfg("sgd", lr=1e-4, target_period=3, seed=5)
    for k in (1, 4, 3, 19):      # 19: two 8-step prefetching graphs + singles
        nets[0].step_pipelined(cfg, k)
        nets[1].step_graph(cfg, k)
    for n in nets:
        n.synchronize()
    a, b = nets
    np.testing.assert_array_equal(a.read_indices(), b.read_indices())
    for x, y in zip(a.read_minibatch(), b.read_minibatch()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.get_flat(0), b.get_flat(0))
    np.testing.assert_array_equal(a.get_flat(1), b.get_flat(1))


def test_rccl_world1_allreduce_and_step(ddq, ref):
    """RCCL plumbing on one GPU: a 1-rank communicator all-reduce is the
    identity, and the fused step with allreduce=1 equals the step without."""
    S, B, N = 16, 8, 64
    rng = np.random.default_rng(2)
    nets = [ddq.DeepQNet(batch=B, frame=S) for _ in range(2)]
    theta = ref.flatten(ref.init_params(S, seed=9))
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    for n in nets:
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(st, rng.integers(0, 4, N).astype(np.uint8) * 0,
                        np.zeros(N, np.int16), np.ones(N, np.uint8), 0, N)
    uid = ddq.DeepQNet.comm_unique_id()
    nets[0].comm_init(uid, 1, 0)
    g = rng.normal(0, 1, theta.size).astype(np.float32)
    nets[0].set_grads_flat(g)
    nets[0].allreduce_grads()
    np.testing.assert_array_equal(nets[0].get_grads_flat(), g)
    for i, n in enumerate(nets):
        cfg = n.step_cfg("sgd", lr=1e-3, target_period=10, allreduce=(i == 0), seed=5)
        n.step_graph(cfg, 3)
        n.synchronize()
    np.testing.assert_array_equal(nets[0].get_flat(0), nets[1].get_flat(0))


@pytest.mark.parametrize("rule,B", [("rmsprop", 16), ("adagrad", 16), ("momentum", 16),
                                    ("rmsprop", 32), ("rmsprop", 100)])
def test_fused_apply_matches_separate_apply(ddq, ref, rule, B):
    """The fused fc4-weight apply (slab-reduce launch, draw counter advanced by
    the head kernel; exchange-free steps) against the separate apply launch
    the exchanges use (a one-member in-process group with the all-reduce
    exchange: sum of one slice, then the plain apply): identical parameters,
    optimizer state and P<-Q syncs over eager, pipelined and graph chains that
    cross sync steps.  B = 100: the fc4 chain's four image chunks, their
    partial sums reduced in the weight-gradient launch."""
    S, N = 16, 300
    rng = np.random.default_rng(31)
    theta = ref.flatten(ref.init_params(S, seed=8))
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    acts = rng.integers(0, 4, N).astype(np.uint8)
    rws = rng.integers(-1, 2, N).astype(np.int16)
    nts = (rng.random(N) > 0.1).astype(np.uint8)
    nets = []
    for _ in range(2):
        n = ddq.DeepQNet(batch=B, frame=S)
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(st, acts, rws, nts, 0, N)
        nets.append(n)
    a, b = nets
    cfg = a.step_cfg(rule, lr=1e-4, target_period=3, seed=9)
    a.step(cfg)
    a.step_pipelined(cfg, 9)
    a.step_graph(cfg, 4)
    a.synchronize()
    grp = ddq.DeepQNet.group_init([b])
    gcfg = b.step_cfg(rule, lr=1e-4, target_period=3, seed=9, exchange="allreduce")
    for _ in range(14):
        ddq.DeepQNet.group_step([b], gcfg, grp)
    b.synchronize()
    np.testing.assert_array_equal(a.read_indices(), b.read_indices())
    np.testing.assert_array_equal(a.get_flat(0), b.get_flat(0))
    np.testing.assert_array_equal(a.get_flat(1), b.get_flat(1))
    np.testing.assert_array_equal(a.optimizer_state(), b.optimizer_state())
    np.testing.assert_array_equal(a.get_grads_flat(), b.get_grads_flat())
    assert not np.array_equal(a.get_flat(0), theta)


@pytest.mark.parametrize("S,rule,lr,frames", [(16, "rmsprop", 1e-4, "random"),
                                               (64, "sgd", 1e-5, "random"),
                                               (64, "rmsprop", 1e-4, "snake")])
def test_no_grad_store_keeps_the_update(ddq, ref, S, rule, lr, frames):
    """DDQ_STEP_NO_GRAD_STORE (exchange-free steps do not store fc4's weight
    gradient; bench --no-grad-store) against the default: identical indices,
    parameters of both towers and optimizer state, bit for bit, over eager,
    pipelined and graph chains across P<-Q syncs; the gradient buffer's conv,
    bias and Q_out blocks equal too, only fc4's weight block is left stale."""
    from ddq.params import init_params_flat
    B, N = 32, 300
    rng = np.random.default_rng(41)
    theta = init_params_flat(S, seed=42)          # the bench's initialisation: live ReLUs
    if frames == "snake":   # the bench's replay contents (bench.py fill_replay)
        from ddq.expgain import synthetic_transitions
        st, acts, rws, nts = synthetic_transitions(N, S, seed=1000)
        nts = np.asarray(nts).astype(np.uint8)
    else:
        st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
        acts = rng.integers(0, 4, N).astype(np.uint8)
        rws = rng.integers(-1, 2, N).astype(np.int16)
        nts = (rng.random(N) > 0.1).astype(np.uint8)
    nets = []
    for _ in range(2):
        n = ddq.DeepQNet(batch=B, frame=S)
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(N)
        n.replay_import(st, acts, rws, nts, 0, N)
        nets.append(n)
    # (64x64 on a small random ring: sgd at a small rate -- lagged rmsprop
    # from c = g^2 diverges there within a few steps, as the reference's rule
    # does, and dead ReLUs would leave nothing to compare; on the bench's Snake
    # frames rmsprop stays live)
    for n, store in zip(nets, (True, False)):
        cfg = n.step_cfg(rule, lr=lr, target_period=3, seed=4, store_grads=store)
        n.step(cfg)
        n.step_pipelined(cfg, 9)
        n.step_graph(cfg, 5)
        n.synchronize()
    a, b = nets
    assert np.isfinite(float(a.blob("loss")))
    np.testing.assert_array_equal(a.read_indices(), b.read_indices())
    np.testing.assert_array_equal(a.get_flat(0), b.get_flat(0))
    np.testing.assert_array_equal(a.get_flat(1), b.get_flat(1))
    np.testing.assert_array_equal(a.optimizer_state(), b.optimizer_state())
    _, off, cnt = a.layout["Qfc4"][0]
    ga, gb = a.get_grads_flat(), b.get_grads_flat()
    keep = np.ones(ga.size, bool)
    keep[off:off + cnt] = False
    np.testing.assert_array_equal(ga[keep], gb[keep])
    assert np.count_nonzero(ga[~keep]) > cnt // 100     # a's last fc4 gradient, stored
    if S == 16:   # the small-map step stores it regardless (K4's apply reads it)
        np.testing.assert_array_equal(ga[~keep], gb[~keep])
    else:
        assert not np.array_equal(ga[~keep], gb[~keep])
