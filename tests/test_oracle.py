"""CPU tests: pin the oracle against the reference's own fixtures / published
numbers, cross-check the two oracle restatements (numpy float64, C fp32)
against an independent torch-CPU float64 implementation."""
import ctypes
import os

import numpy as np
import pytest

from oracle import ref_numpy as ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")

# results/cost-vs-image-size-trials.txt column 6 (128 px: 8,485,668; the
# summary file's 8,484,668 is a typo)
PUBLISHED_PARAMS = {16: 228132, 24: 391972, 32: 621348, 40: 916260, 48: 1276708,
                    56: 1702692, 64: 2194212, 72: 2751268, 80: 3373860, 88: 4061988,
                    96: 4815652, 104: 5634852, 112: 6519588, 120: 7469860, 128: 8485668}
# message size in MB (column 2): 4 bytes per Q parameter (+ a small header)
PUBLISHED_MSG_MB = {16: 0.91, 32: 2.49, 64: 8.78, 128: 33.94}


@pytest.mark.parametrize("S", sorted(PUBLISHED_PARAMS))
def test_param_count_pinned_by_reference_results(S):
    assert ref.num_params(S) == PUBLISHED_PARAMS[S]


@pytest.mark.parametrize("S", sorted(PUBLISHED_MSG_MB))
def test_gradient_message_size_matches_published(S):
    p = ref.init_params(S, seed=0)
    msg = ref.create_message_ref(p, 0)
    assert round(len(msg) / 1e6, 2) == pytest.approx(PUBLISHED_MSG_MB[S], abs=0.011)


def _replay_fixtures():
    return sorted(f for f in os.listdir(GOLD) if f.startswith("replay_"))


@pytest.mark.parametrize("name", _replay_fixtures())
def test_replay_oracle_pinned_by_reference(name):
    f = np.load(os.path.join(GOLD, name))
    r = ref.ReplayRef((4, int(f["S"]), int(f["S"])), int(f["N"]))
    r.state, r.action, r.reward = f["st"], f["action"], f["reward"]
    r.non_terminal, r.head, r.valid = f["non_terminal"], int(f["head"]), int(f["valid"])
    B = int(f["B"])
    if str(f["error"]):
        with pytest.raises(ValueError, match="Can't draw sample of size %d" % B):
            ref.draw_indices(np.random.default_rng(0), r.valid, r.head, B)
        return
    out = r.gather(f["idx"])
    for got, key in zip(out, ("out_state", "out_action", "out_reward", "out_next_state",
                              "out_non_terminal")):
        np.testing.assert_array_equal(got, f[key])
    assert (r.head - 1) not in f["idx"]


def test_replay_ring_semantics():
    """replay.py:70-92: terminal leaves the slot stale; head wraps; valid saturates."""
    r = ref.ReplayRef((4, 2, 2), 3)
    s = lambda v: np.full((4, 2, 2), v, np.uint8)
    r.add_experience(0, 1, s(1))
    r.add_experience(1, 0, None)
    assert (r.head, r.valid) == (2, 2) and r.state[1].max() == 0 and not r.non_terminal[1]
    r.add_experience(2, -1, s(3))
    r.add_experience(3, 1, None)
    assert (r.head, r.valid) == (1, 3)
    assert r.state[0].max() == 1 and not r.non_terminal[0] and r.action[0] == 3


def test_expgain_pinned_by_reference():
    from ddq import expgain
    from ddq.snake import gray_scale
    f = np.load(os.path.join(GOLD, "expgain.npz"))
    for it, e in zip(f["iters"], f["epsilon"]):
        assert expgain.epsilon(int(it)) == pytest.approx(float(e), abs=0)
        assert ref.epsilon(int(it)) == pytest.approx(float(e), abs=0)
    np.testing.assert_array_equal(gray_scale(f["boards"]), f["gray"])
    for S in (16, 24, 64):
        pre = expgain.generate_preprocessor((S, S), gray_scale)
        for b, z in zip(f["boards"], f["zoom%d" % S]):
            np.testing.assert_array_equal(pre(b), z)


# ------------------------------------------------------------------ network
def torch_full_pass(pQ, pP, st, act, rw, ns, nt):
    """Independent float64 implementation on torch CPU autograd."""
    import torch
    import torch.nn.functional as F
    t = lambda a: torch.tensor(np.asarray(a, np.float64))

    def tower(x, p, pre):
        h = x
        for name, pad in (("conv1", 3), ("conv2", 2), ("conv3", 1)):
            W, b = p[pre + name]
            h = F.max_pool2d(F.relu(F.conv2d(h, W, b.reshape(-1), padding=pad)), 2, 2)
        h = h.reshape(h.shape[0], -1)
        W4, b4 = p[pre + "fc4"]
        h = F.relu(h @ W4.reshape(512, -1).T + b4.reshape(-1))
        W5, b5 = p[pre + "_out"]
        return h @ W5.reshape(4, -1).T + b5.reshape(-1)

    qp = {k: [t(w).requires_grad_(True) for w in v] for k, v in pQ.items()}
    pp = {k: [t(w) for w in v] for k, v in pP.items()}
    B = st.shape[0]
    Q = tower(t(st), qp, "Q")
    P = tower(t(ns), pp, "P")
    a = t(act).reshape(B, 4)
    qsa = (Q * a).sum(1)
    y = 0.85 * P.max(1).values * t(nt).reshape(B) + t(rw).reshape(B)
    loss = ((qsa - y.detach()) ** 2).sum() / B / 2
    loss.backward()
    grads = {k: [w.grad.numpy() for w in v] for k, v in qp.items()}
    return float(loss.detach()), Q.detach().numpy(), grads


def random_case(S, B, seed, sparse=False):
    rng = np.random.default_rng(seed)
    pQ = ref.init_params(S, seed=seed, prefix="Q")
    pP = ref.init_params(S, seed=seed + 1, prefix="P")
    for p in (pQ, pP):
        for k in p:
            p[k][0] = (p[k][0] * 3).astype(np.float32)
            p[k][1] = rng.normal(0, 0.05, p[k][1].shape).astype(np.float32)
    if sparse:
        vals = np.array([0, 200, 255], np.float32)
        st = rng.choice(vals, (B, 4, S, S), p=[0.9, 0.08, 0.02])
        ns = rng.choice(vals, (B, 4, S, S), p=[0.9, 0.08, 0.02])
    else:
        st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
        ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    act = np.zeros((B, 4, 1, 1), np.float32)
    act[np.arange(B), rng.integers(0, 4, B)] = 1
    rw = rng.integers(-1, 2, (B, 1, 1, 1)).astype(np.float32)
    nt = (rng.random((B, 1, 1, 1)) > 0.2).astype(np.float32)
    return pQ, pP, st, act, rw, ns, nt


@pytest.mark.parametrize("S,B,sparse", [(16, 4, False), (16, 4, True), (24, 2, False)])
def test_numpy_oracle_matches_torch_float64(S, B, sparse):
    case = random_case(S, B, seed=S + B, sparse=sparse)
    blobs, grads = ref.full_pass(*case)
    tloss, tq, tgrads = torch_full_pass(*case)
    assert blobs["loss"] == pytest.approx(tloss, rel=1e-10)
    np.testing.assert_allclose(blobs["Q_out"], tq, rtol=1e-10, atol=1e-12)
    for k in grads:
        for i in range(2):
            g, tg = grads[k][i].reshape(-1), tgrads[k][i].reshape(-1)
            np.testing.assert_allclose(g, tg, rtol=1e-9, atol=1e-10 * np.abs(tg).max())


@pytest.fixture(scope="module")
def cpu_lib():
    path = os.path.join(ROOT, "oracle", "libddq_cpu.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(path)
    lib.ddq_cpu_num_params.restype = ctypes.c_long
    return lib


def test_c_oracle_matches_numpy_oracle(cpu_lib):
    S, B = 16, 8
    pQ, pP, st, act, rw, ns, nt = random_case(S, B, seed=5)
    blobs, grads = ref.full_pass(pQ, pP, st, act, rw, ns, nt)
    fp = ctypes.POINTER(ctypes.c_float)
    P = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(fp)
    n = cpu_lib.ddq_cpu_num_params(S)
    assert n == ref.num_params(S)
    thq, thp = ref.flatten(pQ), ref.flatten(pP)
    g = np.zeros(n, np.float32)
    out = np.zeros(2 * B * 4 + 3 * B + 1, np.float32)
    keep = [np.ascontiguousarray(a, np.float32) for a in (thq, thp, st, act, rw, ns, nt)]
    rc = cpu_lib.ddq_cpu_full_pass(B, S, *[k.ctypes.data_as(fp) for k in keep],
                                   ctypes.c_float(0.85), g.ctypes.data_as(fp),
                                   out.ctypes.data_as(fp), 2)
    assert rc == 0
    np.testing.assert_allclose(out[:B * 4], blobs["Q_out"].ravel(), rtol=1e-5, atol=1e-6)
    assert out[-1] == pytest.approx(blobs["loss"], rel=1e-5)
    gref = ref.flatten(grads)
    scale = np.abs(gref).max()
    assert np.max(np.abs(g - gref)) <= 1e-4 * scale


@pytest.mark.parametrize("isa", [512, 256])
@pytest.mark.parametrize("S,B,threads", [(24, 3, 3), (40, 5, 4)])
def test_c_oracle_blocked_gemm_edges(cpu_lib, isa, S, B, threads):
    """The packed SGEMM's ragged edges (HW, K and the batch not multiples of
    the micro-tile) on both micro-kernels, against the numpy oracle."""
    got = cpu_lib.ddq_cpu_set_isa(isa)
    if got != isa:
        pytest.skip("no AVX-512 on this host")
    try:
        pQ, pP, st, act, rw, ns, nt = random_case(S, B, seed=S)
        blobs, grads = ref.full_pass(pQ, pP, st, act, rw, ns, nt)
        fp = ctypes.POINTER(ctypes.c_float)
        n = cpu_lib.ddq_cpu_num_params(S)
        g = np.zeros(n, np.float32)
        out = np.zeros(2 * B * 4 + 3 * B + 1, np.float32)
        keep = [np.ascontiguousarray(a, np.float32)
                for a in (ref.flatten(pQ), ref.flatten(pP), st, act, rw, ns, nt)]
        rc = cpu_lib.ddq_cpu_full_pass(B, S, *[k.ctypes.data_as(fp) for k in keep],
                                       ctypes.c_float(0.85), g.ctypes.data_as(fp),
                                       out.ctypes.data_as(fp), threads)
        assert rc == 0
        for lo, key in ((0, "Q_out"), (B * 4, "P_out")):   # fp32 sums of ~4.6e3 terms
            r = blobs[key].ravel()
            np.testing.assert_allclose(out[lo:lo + B * 4], r, rtol=1e-5,
                                       atol=5e-6 * np.abs(r).max())
        gref = ref.flatten(grads)
        assert np.max(np.abs(g - gref)) <= 1e-4 * np.abs(gref).max()
    finally:
        cpu_lib.ddq_cpu_set_isa(512)


def test_c_oracle_apply_matches_restatement(cpu_lib):
    rng = np.random.default_rng(0)
    n = 1000
    for rule in (0, 1, 2):
        th = rng.normal(0, 1, n).astype(np.float32)
        th_c = th.copy()
        st_c = np.zeros(n, np.float32)
        state = None
        for step in range(3):
            g = rng.normal(0, 1e-2, n).astype(np.float32)
            fp = ctypes.POINTER(ctypes.c_float)
            cpu_lib.ddq_cpu_apply(rule, ctypes.c_long(n), th_c.ctypes.data_as(fp),
                                  g.ctypes.data_as(fp), st_c.ctypes.data_as(fp), int(step == 0),
                                  ctypes.c_float(1e-3), ctypes.c_float(0.9), ctypes.c_float(1e-8))
            if rule == 0:
                th = ref.sgd_update(th, g, 1e-3)
            elif rule == 1:
                th, state = ref.rmsprop_update(th, g, state, 1e-3)
            else:
                th, state = ref.adagrad_update(th, g, state, 1e-3)
            np.testing.assert_allclose(th_c, th, rtol=1e-6, atol=1e-9)


def test_rmsprop_uses_lagged_cache():
    """server.py:89-105: the update applies the cache from BEFORE this gradient."""
    th = np.ones(2, np.float32)
    g1 = np.array([1.0, 1.0], np.float32)
    th1, c1 = ref.rmsprop_update(th, g1, None, 0.1)
    np.testing.assert_allclose(th1, 1 - 0.1 * 1 / np.sqrt(1 + 1e-8), rtol=1e-6)
    g2 = np.array([2.0, 0.0], np.float32)
    th2, c2 = ref.rmsprop_update(th1, g2, c1, 0.1)
    np.testing.assert_allclose(th2, th1 - 0.1 * g2 / np.sqrt(c1 + 1e-8), rtol=1e-6)
    np.testing.assert_allclose(c2, 0.9 * c1 + 0.1 * g2 ** 2, rtol=1e-6)


def test_magnitudes_bound_every_output():
    """oracle.magnitudes (the per-element sum of |terms| the parity tolerance
    scales with) bounds |value| of every blob and gradient element, and is
    routing-consistent (same result when the oracle's own routing is passed)."""
    S, B = 16, 4
    rng = np.random.default_rng(12)
    pQ, pP = ref.init_params(S, seed=1), ref.init_params(S, seed=2, prefix="P")
    st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    act = np.zeros((B, 4, 1, 1), np.float32)
    act[np.arange(B), rng.integers(0, 4, B)] = 1
    rw = rng.integers(-1, 2, (B, 1, 1, 1)).astype(np.float32)
    nt = np.ones((B, 1, 1, 1), np.float32)
    blobs, grads, cache = ref.full_pass(pQ, pP, st, act, rw, ns, nt, return_cache=True)
    mb, mg = ref.magnitudes(pQ, pP, st, act, rw, ns, nt)
    for k in blobs:
        assert np.all(np.abs(blobs[k]) <= np.asarray(mb[k]) * (1 + 1e-12) + 1e-300), k
    for k in grads:
        for i in range(2):
            assert np.all(np.abs(grads[k][i]) <= mg[k][i] * (1 + 1e-12) + 1e-300), (k, i)
    routes = {i: ref.route_codes(cache["act%d" % i], cache["arg%d" % i]) for i in (1, 2, 3)}
    mb2, mg2 = ref.magnitudes(pQ, pP, st, act, rw, ns, nt, routes=routes)
    for k in grads:
        for i in range(2):
            np.testing.assert_allclose(mg2[k][i], mg[k][i], rtol=1e-12)
