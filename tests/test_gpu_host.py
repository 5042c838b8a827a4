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
    with pytest.raises(ValueError):
        ds.sample_direct(*arrs, 1000)
    # persistence round trip (replay.py:185-192 persists, reopen appends)
    ds.close()
    ds2 = ReplayDataset(str(tmp_path / "d.npz"), (4, S, S), dset_size=N, batch_size=B)
    assert (ds2.head, ds2.valid) == (r.head, r.valid)
    st, ac, rw, nt = ds2._net.replay_export()
    np.testing.assert_array_equal(st, r.state)
    ds2.close()


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


def test_barista_tcp_loop_with_dummy_client(param_server, tmp_path, monkeypatch):
    """Config 1 plumbing: dummy client -> Barista TCP 'G' -> param server."""
    from ddq.barista import main as bmain
    from ddq.barista.dummy_client import DummyClient
    ps, driver = param_server
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
