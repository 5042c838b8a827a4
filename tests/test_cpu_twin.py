"""The CPU-mode twin libddq_cpu.so (distributed-deep-q_amd/cpu/twin.cpp): the
reference's Caffe CPU mode (main.py:128,149-151 ``--mode cpu``; BASELINE.json
configs[0], "deepq16 Snake DQN, Caffe CPU mode, single Barista worker driven by
barista.dummy_client (plumbing, no GPU)").  No GPU is needed: these run in the
CPU suite.  The twin is product code written for this library (it neither
links nor calls oracle/); the oracle is the checker here, as in the GPU tests.

* every symbol of include/ddq_hip.h is exported; GPU-only calls refuse with
  DDQ_ESTATE;
* full pass (blobs, every Q gradient) against the float64 oracle within rtol
  1e-4 + 2e-7 * (sum of |terms|) (tests/_parity.py), pool routing adopted only
  at proven near-ties;
* the update rules against server.py's (oracle restatement);
* the replay gather bit-exact against the reference's own replay.py fixtures;
* config 1 end to end: dummy client -> Barista TCP 'G' -> HTTP param server,
  worker and server both in CPU mode, every pushed gradient checked.
"""
import glob
import os
import re
import subprocess
import threading
import time

import numpy as np
import pytest

from _parity import check_full_pass, close
from oracle import ref_numpy as ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HEADER = os.path.join(ROOT, "include", "ddq_hip.h")


@pytest.fixture(scope="module")
def ddq():
    import ddq as m
    from ddq import _lib
    if not os.path.exists(_lib.CPU_LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "distributed-deep-q_amd"),
                        "ddq/_lib/libddq_cpu.so"], check=True)
    return m


def cpu_net(ddq, B, S):
    return ddq.DeepQNet(batch=B, frame=S, mode="cpu")


def test_exports_every_header_symbol(ddq):
    from ddq import _lib
    lib = _lib.load(mode="cpu")
    names = set(re.findall(r"\b(ddq_[a-z0-9_]+)\s*\(", open(HEADER).read()))
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.CPU_LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T ddq_" in ln}
    assert names == exported
    assert lib.ddq_abi_version() == _lib.ABI_VERSION


def test_gpu_only_calls_refuse(ddq):
    from ddq import _lib
    net = cpu_net(ddq, 4, 16)
    net.replay_create(64)
    cfg = net.step_cfg("rmsprop")
    for call in (lambda: net.step(cfg), lambda: net.step_graph(cfg, 2),
                 lambda: net.replay_sample_device(1), lambda: net.index_log_enable(4)):
        with pytest.raises(_lib.DDQError) as ei:
            call()
        assert ei.value.code == _lib.DDQ_ESTATE and "CPU mode" in ei.value.msg
    assert net.small_path() == (False, "CPU mode")
    net.close()


def make_inputs(rng, B, S, frames):
    if frames == "uniform":
        st = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
        ns = rng.integers(0, 256, (B, 4, S, S)).astype(np.float32)
    else:                     # snake-like sparse frames {0, 200, 255}
        st = rng.choice(np.array([0, 200, 255], np.float32), (B, 4, S, S), p=[0.9, 0.08, 0.02])
        ns = rng.choice(np.array([0, 200, 255], np.float32), (B, 4, S, S), p=[0.9, 0.08, 0.02])
    act = np.zeros((B, 4, 1, 1), np.float32)
    act[np.arange(B), rng.integers(0, 4, B)] = 1
    rw = rng.integers(-1, 2, (B, 1, 1, 1)).astype(np.float32)
    nt = (rng.random((B, 1, 1, 1)) > 0.2).astype(np.float32)
    return st, act, rw, ns, nt


@pytest.mark.parametrize("S,B,frames", [(16, 4, "snake"), (16, 8, "uniform"), (24, 2, "snake")])
def test_full_pass_parity(ddq, S, B, frames):
    rng = np.random.default_rng(500 + S + B)
    pQ = ref.init_params(S, seed=7, prefix="Q")
    pP = ref.init_params(S, seed=8, prefix="P")
    for p in (pQ, pP):                       # activations O(1), no dead towers
        for k in p:
            p[k][0] = (p[k][0] * 3).astype(np.float32)
            p[k][1] = rng.normal(0, 0.05, p[k][1].shape).astype(np.float32)
    net = cpu_net(ddq, B, S)
    params = dict(pQ)
    params.update(pP)
    net.set_params(params)
    mb = make_inputs(rng, B, S, frames)
    net.write_minibatch(*mb)
    loss = net.forward_backward()
    check_full_pass(ref, net, pQ, pP, mb)
    assert loss == float(net.blob("loss"))
    np.testing.assert_array_equal(net.read_minibatch()[0], mb[0])
    net.close()


@pytest.mark.parametrize("rule", ["sgd", "rmsprop", "adagrad", "momentum"])
def test_apply_rules(ddq, rule):
    S = 16
    rng = np.random.default_rng(11)
    net = cpu_net(ddq, 8, S)
    theta = ref.flatten(ref.init_params(S, seed=3))
    net.set_flat(0, theta)
    net.reset_optimizer()
    P = theta.size
    is_bias = np.zeros(P, bool)
    for blobs in net.layout.values():
        s, o, c = blobs[1]
        is_bias[o:o + c] = True
    th, state = theta.copy(), None
    for step in range(3):
        g = rng.normal(0, 1e-2, P).astype(np.float32)
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
    net.close()


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "replay_*.npz"))))
def test_replay_gather_bitexact_vs_reference(ddq, path):
    from ddq import _lib
    f = np.load(path)
    S, N, B = int(f["S"]), int(f["N"]), int(f["B"])
    net = cpu_net(ddq, B, S)
    net.replay_create(N)
    net.replay_import(f["st"], f["action"], f["reward"], f["non_terminal"].astype(np.uint8),
                      int(f["head"]), int(f["valid"]))
    if str(f["error"]):
        with pytest.raises(_lib.DDQError) as ei:
            net.replay_sample(np.arange(B, dtype=np.int32))
        assert "Can't draw sample of size %d from replay dataset of size %d" % (
            B, int(f["valid"])) in str(ei.value)
        return
    net.replay_sample(f["idx"])
    st, ac, rw, ns, nt = net.read_minibatch()
    np.testing.assert_array_equal(st, f["out_state"])
    np.testing.assert_array_equal(ns, f["out_next_state"])
    np.testing.assert_array_equal(ac.reshape(f["out_action"].shape), f["out_action"])
    np.testing.assert_array_equal(rw.reshape(f["out_reward"].shape), f["out_reward"])
    np.testing.assert_array_equal(nt.reshape(f["out_non_terminal"].shape), f["out_non_terminal"])
    net.close()


def test_select_action_first_max(ddq):
    S, B = 16, 8
    rng = np.random.default_rng(4)
    pQ = ref.init_params(S, seed=5, prefix="Q")
    for k in pQ:
        pQ[k][0] = (pQ[k][0] * 3).astype(np.float32)
    net = cpu_net(ddq, B, S)
    net.set_flat(0, ref.flatten(pQ))
    states = rng.integers(0, 256, (B, 4, S, S)).astype(np.uint8)
    got = net.select_action(states)
    q = ref.net_forward(states.astype(np.float64), {k: [np.asarray(w, np.float64) for w in v]
                                                     for k, v in pQ.items()}, "Q")["out"]
    for b in range(B):   # first max unless the float64 values tie within fp32 rounding
        top = np.flatnonzero(q[b] >= q[b].max() - 1e-6 * np.abs(q[b]).max())
        assert got[b] in top
    net.close()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_config1_barista_tcp_loop_cpu_mode(tmp_path, monkeypatch):
    """Config 1 without a GPU: the dummy client sends 'G' three times to a
    Barista worker in CPU mode (main.py --mode cpu), which acts through the CPU
    Q tower, samples its replay, runs the full pass and pushes the gradient to
    an HTTP param server in CPU mode; every pushed gradient against the
    oracle's full pass on the parameters and minibatch the worker held, the
    server's model after the pushes against the oracle's rmsprop chain."""
    from ddq.barista import main as bmain
    from ddq.barista.baristanet import BaristaNet
    from ddq.barista.dummy_client import DummyClient
    from ddq.param_server import ParamServer
    ps = ParamServer(frame=16, batch=32, update="rmsprop", lr=1e-3, special_update=2, mode="cpu")
    ps.init_params(seed=11)
    sport = free_port()
    sth = threading.Thread(target=ps.serve, kwargs={"port": sport}, daemon=True)
    sth.start()
    time.sleep(0.3)
    try:
        theta0 = ps.net.get_flat(0)
        pushes, errors = [], []
        orig = BaristaNet.send_gradient_update

        def checked_push(self):
            try:
                dq, S = self.dqn, self.dqn.frame
                assert dq.mode == "cpu"
                pQ, pP = dq.get_flat(0), dq.get_flat(1)
                check_full_pass(ref, dq, ref.unflatten(pQ, S, "Q"), ref.unflatten(pP, S, "P"),
                                dq.read_minibatch(), quiet=True, what="push%d " % len(pushes))
                pushes.append(dq.get_grads_flat())
            except Exception as e:                 # raised again in the test's thread
                errors.append(e)
            return orig(self)
        monkeypatch.setattr(BaristaNet, "send_gradient_update", checked_push)
        monkeypatch.chdir(tmp_path)
        port = free_port()
        args = [os.path.join(GOLD, "deepq16.prototxt"), "none", "--mode", "cpu", "--port",
                str(port), "--driver", "127.0.0.1:%d" % sport, "--dataset",
                str(tmp_path / "replay.npz"), "--dset-size", "300", "--initial-replay", "120",
                "--overwrite", "--max-requests", "3"]
        th = threading.Thread(target=bmain.main, args=(args,), daemon=True)
        th.start()
        flag = tmp_path / "flags" / ("__BARISTA_READY__.%d" % port)
        for _ in range(1200):
            if flag.exists():
                break
            time.sleep(0.1)
        assert flag.exists()
        for _ in range(3):
            c = DummyClient("127.0.0.1", port)
            c.send(b"G")
            assert c.recv() == b"Updated"
            c.close()
        th.join(timeout=120)
        assert ps.iteration == 3
        if errors:
            raise errors[0]
        assert len(pushes) == 3
        theta, cache = theta0, None
        for g in pushes:
            theta, cache = ref.rmsprop_update(theta, g, cache, 1e-3)
        np.testing.assert_allclose(ps.net.get_flat(0), theta, rtol=1e-5, atol=1e-8)
    finally:
        ps.shutdown()
