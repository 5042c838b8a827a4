"""GPU tests of the host drop-ins: ReplayDataset, BaristaNet, ParamServer,
the Barista TCP loop + dummy client (BASELINE config 1 plumbing)."""
import os
import random
import socket
import threading
import time

import numpy as np
import pytest

from oracle import ref_numpy as ref

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_replay_dataset_dropin_matches_oracle(tmp_path):
    from ddq.replay import ReplayDataset
    S, N, B = 16, 50, 8
    rng = np.random.default_rng(0)
    ds = ReplayDataset(str(tmp_path / "d.npz"), (4, S, S), dset_size=N, overwrite=True,
                       batch_size=B)
    r = ref.ReplayRef((4, S, S), N)
    for i in range(70):
        st = None if i % 9 == 8 else rng.integers(0, 256, (4, S, S)).astype(np.uint8)
        a, rw = int(rng.integers(0, 4)), int(rng.integers(-1, 2))
        ds.add_experience(a, rw, st)
        r.add_experience(a, rw, st)
    assert (ds.head, ds.valid) == (r.head, r.valid)
    arrs = [np.zeros((B, 4, S, S), np.float32), np.zeros((B, 4, 1, 1), np.float32),
            np.zeros((B, 1, 1, 1), np.float32), np.zeros((B, 4, S, S), np.float32),
            np.zeros((B, 1, 1, 1), np.float32)]
    random.seed(3)
    ds.sample_direct(*arrs, B)
    random.seed(3)
    idx = ds.draw_indices(B)
    exp = r.gather(idx)
    for got, want in zip(arrs, exp):
        np.testing.assert_array_equal(got, want)
    # any sample size, as the reference's caller arrays allow (replay.py:144-183)
    for n in (1, 3, 20):
        out = [np.zeros((n, 4, S, S), np.float32), np.zeros((n, 4, 1, 1), np.float32),
               np.zeros((n, 1, 1, 1), np.float32), np.zeros((n, 4, S, S), np.float32),
               np.zeros((n, 1, 1, 1), np.float32)]
        random.seed(10 + n)
        ds.sample_direct(*out, n)
        random.seed(10 + n)
        exp = r.gather(ds.draw_indices(n))
        for got, want in zip(out, exp):
            np.testing.assert_array_equal(got, want)
    with pytest.raises(ValueError):
        ds.sample_direct(*arrs, 1000)
    # persistence round trip (replay.py:185-192 persists, reopen appends)
    ds.close()
    ds2 = ReplayDataset(str(tmp_path / "d.npz"), (4, S, S), dset_size=N, batch_size=B)
    assert (ds2.head, ds2.valid) == (r.head, r.valid)
    st, ac, rw, nt = ds2._net.replay_export()
    np.testing.assert_array_equal(st, r.state)
    ds2.close()


def test_replay_dataset_resumes_reference_files(tmp_path):
    """F1: the drop-in opens files the reference's replay.py persisted
    (fixtures: oracle/gen_hdf5_golden.py), gathers exactly what the reference
    gathered from them, and persists a file that reads back identically."""
    import shutil
    from ddq import h5lite
    from ddq.replay import ReplayDataset
    S = 16
    want = np.load(os.path.join(GOLD, "h5_ref_s16.npz"))
    p = str(tmp_path / "ref.hdf5")
    shutil.copy(os.path.join(GOLD, "h5_ref_s16.hdf5"), p)
    ds = ReplayDataset(p, (4, S, S), dset_size=12, batch_size=4)
    assert (ds.head, ds.valid) == (int(want["head"]), int(want["valid"]))
    st, ac, rw, nt = ds._net.replay_export()
    for got, k in ((st, "state"), (ac, "action"), (rw, "reward"), (nt, "non_terminal")):
        np.testing.assert_array_equal(got, want[k], err_msg=k)
    ds.close()

    f = np.load(os.path.join(GOLD, "h5_resume.npz"))
    p = str(tmp_path / "resume.hdf5")
    shutil.copy(os.path.join(GOLD, "h5_resume_out.hdf5"), p)
    B = len(f["idx"])
    ds = ReplayDataset(p, (4, S, S), dset_size=10, batch_size=B)
    assert (ds.head, ds.valid) == (int(f["fin_head"]), int(f["fin_valid"]))
    ds.draw_indices = lambda n: [int(i) for i in f["idx"]]     # the reference's scripted draw
    out = [np.zeros((B, 4, S, S), np.float32), np.zeros((B, 4, 1, 1), np.float32),
           np.zeros((B, 1, 1, 1), np.float32), np.zeros((B, 4, S, S), np.float32),
           np.zeros((B, 1, 1, 1), np.float32)]
    ds.sample_direct(*out, B)
    for got, k in zip(out, ("state", "action", "reward", "next_state", "non_terminal")):
        np.testing.assert_array_equal(got, f["out_" + k], err_msg=k)
    ds.close()                                   # persists (replay.py:185-192)
    got = h5lite.read_replay(p)
    for k in ("state", "action", "reward", "non_terminal", "head", "valid"):
        np.testing.assert_array_equal(got[k], f["fin_" + k], err_msg=k)


def test_policy_evaluator_and_q_convergence_match_oracle(tmp_path):
    """F4: evaluation.py's greedy evaluation (batched select_action on the
    GPU) scores exactly what the float64 oracle's action choices score, and
    q_convergence's mean Q_out matches the oracle forward on the same draws."""
    from ddq import evaluation
    from ddq.barista.baristanet import BaristaNet
    from ddq.replay import ReplayDataset
    from ddq.expgain import synthetic_transitions

    class OracleNet:
        def __init__(self, B, S, pQ):
            self.batch_size, self.pQ = B, pQ
            self.state = np.zeros((B, 4, S, S), np.float32)

        def select_action(self, states, batch_size=1):
            return ref.select_action(np.asarray(states, np.float32), self.pQ)

    S = 16
    net = BaristaNet(os.path.join(GOLD, "deepq16.prototxt"), None, None)
    B = net.batch_size
    pQ = ref.init_params(S, seed=21)
    gpu = evaluation.PolicyEvaluator(None, None, net=net, seed=9, max_moves=300)
    cpu = evaluation.PolicyEvaluator(None, None, net=OracleNet(B, S, pQ), seed=9, max_moves=300)
    assert gpu.evaluate(pQ, 40) == cpu.evaluate(None, 40)

    ds = ReplayDataset(str(tmp_path / "q.hdf5"), (4, S, S), dset_size=300, batch_size=B)
    st, ac, rw, nt = synthetic_transitions(300, S, seed=4)
    r = ref.ReplayRef((4, S, S), 300)
    for i in range(300):
        ds.add_experience(int(ac[i]), int(rw[i]), st[i] if nt[i] else None)
        r.add_experience(int(ac[i]), int(rw[i]), st[i] if nt[i] else None)
    net.add_dataset(ds)
    random.seed(13)
    got = evaluation.evaluate_model(net, pQ, 3)
    random.seed(13)
    want = 0.0
    p64 = {k: [np.asarray(w, np.float64) for w in v] for k, v in pQ.items()}
    for _ in range(3):
        x = r.gather(ds.draw_indices(B))[0]
        want += ref.net_forward(np.asarray(x, np.float64), p64, "Q")["out"].mean()
    assert got == pytest.approx(want / 3, rel=1e-4, abs=1e-7)
    ds.close()


@pytest.fixture
def param_server():
    from ddq.param_server import ParamServer
    ps = ParamServer(frame=16, batch=32, update="rmsprop", lr=1e-3, special_update=2)
    ps.init_params(seed=11)
    port = free_port()
    th = threading.Thread(target=ps.serve, kwargs={"port": port}, daemon=True)
    th.start()
    time.sleep(0.3)
    yield ps, "127.0.0.1:%d" % port
    ps.shutdown()


def test_worker_param_server_round_trip(param_server):
    from ddq.barista.baristanet import BaristaNet
    ps, driver = param_server
    net = BaristaNet(os.path.join(GOLD, "deepq16.prototxt"), None, driver)
    theta0 = ps.net.get_flat(0)
    it = net.fetch_model()                       # iteration 0: P <- Q on the server
    assert it == 0
    np.testing.assert_array_equal(net.dqn.get_flat(0), theta0)
    np.testing.assert_array_equal(net.dqn.get_flat(1), theta0)
    np.random.seed(0)
    net.dummy_load_minibatch()
    net.full_pass()
    g = net.dqn.get_grads_flat()
    assert net.send_gradient_update() == b"Updated"
    assert ps.iteration == 1
    th_ref, _ = ref.rmsprop_update(theta0, g, None, 1e-3)
    np.testing.assert_allclose(ps.net.get_flat(0), th_ref, rtol=1e-6, atol=1e-9)
    # second pull at iteration 1: no target sync; P stays theta0
    net.fetch_model()
    np.testing.assert_array_equal(net.dqn.get_flat(0), ps.net.get_flat(0))
    np.testing.assert_array_equal(net.dqn.get_flat(1), theta0)


def test_partial_gradient_message_is_refused(param_server):
    """A gradient message lacking Q blobs is refused (the device apply would
    otherwise decay the rmsprop cache of the missing blobs); the server state
    is untouched and the HTTP route answers 400."""
    import urllib.request
    from ddq.barista import messaging
    ps, driver = param_server
    theta0 = ps.net.get_flat(0)
    p = ref.init_params(16, seed=4)
    del p["Qconv2"]
    msg = messaging.create_net_message(p, "diff")
    with pytest.raises(ValueError, match="Qconv2"):
        ps.update_params(msg)
    req = urllib.request.Request("http://%s/api/v1/update_model" % driver, data=msg,
                                 headers={"Content-Type": "application/deepQ"})
    with pytest.raises(urllib.error.HTTPError) as ei:
        urllib.request.urlopen(req, timeout=10)
    assert ei.value.code == 400
    assert ps.iteration == 0
    np.testing.assert_array_equal(ps.net.get_flat(0), theta0)


def test_barista_tcp_loop_with_dummy_client(param_server, tmp_path, monkeypatch):
    """Config 1: dummy client -> Barista TCP 'G' -> param server, checked by
    value: every gradient the worker pushes against the oracle's full pass on
    the parameters and minibatch the worker held (GPU routing at proven
    near-ties, tests/_parity.py), and the server's model after the three
    pushes against the oracle's rmsprop chain over the pushed gradients
    (server.py:86-105, first call c = g^2, then the lagged cache)."""
    from _parity import check_full_pass
    from ddq.barista import main as bmain
    from ddq.barista.baristanet import BaristaNet
    from ddq.barista.dummy_client import DummyClient
    ps, driver = param_server
    theta0 = ps.net.get_flat(0)
    pushes, errors = [], []
    orig = BaristaNet.send_gradient_update

    def checked_push(self):
        try:
            dq, S = self.dqn, self.dqn.frame
            pQ, pP = dq.get_flat(0), dq.get_flat(1)
            check_full_pass(ref, dq, ref.unflatten(pQ, S, "Q"), ref.unflatten(pP, S, "P"),
                            dq.read_minibatch(), quiet=True, what="push%d " % len(pushes))
            pushes.append(dq.get_grads_flat())
        except Exception as e:                     # raised again in the test's thread
            errors.append(e)
        return orig(self)
    monkeypatch.setattr(BaristaNet, "send_gradient_update", checked_push)
    monkeypatch.chdir(tmp_path)
    port = free_port()
    args = ["%s" % os.path.join(GOLD, "deepq16.prototxt"), "none", "--port", str(port),
            "--driver", driver, "--dataset", str(tmp_path / "replay.npz"), "--dset-size", "300",
            "--initial-replay", "120", "--overwrite", "--max-requests", "3"]
    th = threading.Thread(target=bmain.main, args=(args,), daemon=True)
    th.start()
    flag = tmp_path / "flags" / ("__BARISTA_READY__.%d" % port)
    for _ in range(600):
        if flag.exists():
            break
        time.sleep(0.1)
    assert flag.exists()
    for i in range(3):
        c = DummyClient("127.0.0.1", port)
        c.send(b"G")
        assert c.recv() == b"Updated"
        c.close()
    th.join(timeout=60)
    assert ps.iteration == 3
    if errors:
        raise errors[0]
    assert len(pushes) == 3
    theta, cache = theta0, None
    for g in pushes:
        theta, cache = ref.rmsprop_update(theta, g, cache, 1e-3)
    np.testing.assert_allclose(ps.net.get_flat(0), theta, rtol=1e-5, atol=1e-8)


def test_time_layer_times_the_step_kernels_without_side_effects():
    """ddq_time_layer (the bench's roofline timing) relaunches one forward conv
    layer of the step: positive times, the next full pass unchanged, and an
    unknown layer name is an error, not a launch."""
    import ddq
    S, B = 16, 32
    rng = np.random.default_rng(7)
    net = ddq.DeepQNet(batch=B, frame=S, device=0)
    theta = ref.flatten(ref.init_params(S, seed=2))
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    ac = np.eye(4, dtype=np.float32)[rng.integers(0, 4, B)].reshape(B, 4, 1, 1)
    rw = rng.integers(-1, 2, (B, 1, 1, 1)).astype(np.float32)
    nt = np.ones((B, 1, 1, 1), np.float32)
    net.write_minibatch(st, ac, rw, ns, nt)
    loss0 = net.forward_backward()
    g0 = net.get_grads_flat()
    for name in ("conv1_fwd", "conv2_fwd", "conv3_fwd"):
        us = net.time_layer(name, 5)
        assert 0.0 < us < 1e5, (name, us)
    with pytest.raises(Exception):
        net.time_layer("fc9_fwd", 1)
    loss1 = net.forward_backward()
    assert loss1 == loss0
    np.testing.assert_array_equal(net.get_grads_flat(), g0)
    net.close()
