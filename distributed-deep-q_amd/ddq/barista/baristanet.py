"""BaristaNet: the worker's network wrapper (barista/baristanet.py, reference)
with the same constructor and methods, computing on the MI355X.

``BaristaNet(architecture, model, driver, dataset=None, logpath=None,
reset_log=False)``:
* ``architecture`` -- the deepq ``train_val.prototxt`` (its MEMORY_DATA dims and
  the target coefficient are read from the text; the layer graph itself is the
  fixed deepq network implemented in libddq_hip.so) or a dict
  ``{"batch": B, "frame": S, "gamma": g}``;
* ``model`` -- ``.npz`` file of {name: W, name + "/1": b} blobs, or None for the
  prototxt fillers;
* ``driver`` -- "host:port" of the parameter server, or None (dummy pull/push,
  baristanet.py:99-103, :125-133).

The input buffers ``state``, ``action``, ``reward``, ``next_state``,
``non_terminal`` have the reference's shapes (baristanet.py:30-34).  They are
bound to the device minibatch (the MEMORY_DATA zero-copy binding,
baristanet.py:41-43): ``load_minibatch`` gathers straight into device memory,
and ``sync_inputs()`` / ``push_inputs()`` move them host <-> device on demand.
"""
from __future__ import annotations

import os
import re
import urllib.request

import numpy as np

from ..net import DeepQNet, GAMMA
from .. import params as P
from . import messaging


def parse_architecture(architecture):
    """Batch/frame/gamma of a deepq prototxt (train_val.prototxt:2-37, :465-476)."""
    if isinstance(architecture, dict):
        return (int(architecture.get("batch", 32)), int(architecture.get("frame", 16)),
                float(architecture.get("gamma", GAMMA)))
    with open(architecture) as fp:
        txt = fp.read()
    m = re.search(r"memory_data_param\s*:?\s*\{([^}]*)\}", txt)
    if not m:
        raise ValueError("no MEMORY_DATA layer in %s" % architecture)
    body = m.group(1)
    get = lambda key: int(re.search(r"%s\s*:\s*(\d+)" % key, body).group(1))
    batch, channels, h, w = get("batch_size"), get("channels"), get("height"), get("width")
    if channels != 4 or h != w:
        raise ValueError("deepq expects 4 square frames, got %dx%dx%d" % (channels, h, w))
    gamma = GAMMA
    t = re.search(r'name:\s*"target_Q_sa".*?coeff\s*:\s*([0-9.eE+-]+)', txt, re.S)
    if t:
        gamma = float(t.group(1))
    return batch, h, gamma


class _Blob:
    """pycaffe-like blob view: ``.data`` / ``.diff`` numpy arrays."""

    def __init__(self, data, diff):
        self.data, self.diff = data, diff


class BaristaNet:
    def __init__(self, architecture, model, driver, dataset=None, logpath=None,
                 reset_log=False, device=0, mode="gpu"):
        batch, frame, gamma = parse_architecture(architecture)
        # mode: main.py:149-151 caffe.set_mode_gpu / set_mode_cpu
        self.mode = mode
        self.dqn = DeepQNet(batch=batch, frame=frame, device=device, gamma=gamma, mode=mode)
        if model is not None and os.path.exists(str(model)):
            with np.load(model, allow_pickle=False) as f:
                blobs = {k: f[k] for k in f.files}
            params = {}
            for name in self.dqn.q_names + self.dqn.p_names:
                if name in blobs:
                    params[name] = [blobs[name], blobs[name + "/1"]]
            self.dqn.set_params(params)
        else:
            self.dqn.set_flat(0, P.init_params_flat(frame))
        self.dqn.sync_target()
        self.dataset = None
        self.driver = driver
        # logpath / reset_log: accepted for signature compatibility; the
        # reference's per-step norm logging (netutils.NetLogger) is monitoring,
        # out of scope here
        B, S = batch, frame
        self.state = np.zeros((B, 4, S, S), np.float32)
        self.action = np.zeros((B, 4, 1, 1), np.float32)
        self.reward = np.zeros((B, 1, 1, 1), np.float32)
        self.next_state = np.zeros((B, 4, S, S), np.float32)
        self.non_terminal = np.zeros((B, 1, 1, 1), np.float32)
        self.batch_size = B
        self.iteration = 0
        if dataset is not None:
            self.add_dataset(dataset)

    # ----------------------------------------------------------- net-like API
    @property
    def params(self):
        """OrderedDict name -> [blob(.data, .diff)] (pycaffe ``net.params``)."""
        data = self.dqn.split(self.dqn.get_flat(0), "Q")
        diff = self.dqn.split(self.dqn.get_grads_flat(), "Q")
        out = {k: [_Blob(d, g) for d, g in zip(data[k], diff[k])] for k in data}
        pdata = self.dqn.split(self.dqn.get_flat(1), "P")
        out.update({k: [_Blob(d, np.zeros_like(d)) for d in v] for k, v in pdata.items()})
        return out

    @property
    def blobs(self):
        class _B:
            def __init__(s, a):
                s.data = a
        return {name: _B(self.dqn.blob(name)) for name in
                ("Q_out", "P_out", "Q_sa", "P_sa", "target_Q_sa", "loss")}

    def add_dataset(self, dset):
        dset.attach(self.dqn)
        self.dataset = dset

    # --------------------------------------------------------------- inputs
    def push_inputs(self):
        """Host input arrays -> device minibatch."""
        self.dqn.write_minibatch(self.state, self.action.reshape(self.batch_size, 4),
                                 self.reward, self.next_state, self.non_terminal)

    def sync_inputs(self):
        """Device minibatch -> host input arrays."""
        st, ac, rw, ns, nt = self.dqn.read_minibatch()
        self.state[...], self.action[...], self.reward[...] = st, ac, rw
        self.next_state[...], self.non_terminal[...] = ns, nt

    def load_minibatch(self):
        """baristanet.py:55-68: sample from the replay into the net inputs."""
        if self.dataset:
            idx = self.dataset.draw_indices(self.batch_size)
            self.dqn.replay_sample(np.asarray(idx, np.int32))
        else:
            print("Warning: no dataset specified, using dummy data.")
            self.dummy_load_minibatch()

    def dummy_load_minibatch(self):
        """baristanet.py:70-83: uniform frames, one-hot actions, rewards in [-5,5]."""
        B = self.batch_size
        self.state[...] = np.random.randint(0, 256, size=self.state.shape)
        self.action[...] = 0
        self.action[np.arange(B), np.random.randint(0, 4, size=(B,))] = 1
        self.reward[...] = np.random.randint(-5, 6, size=self.reward.shape)
        self.next_state[...] = np.random.randint(0, 256, size=self.next_state.shape)
        self.non_terminal[...] = np.random.choice([True, False], size=self.non_terminal.shape)
        self.push_inputs()

    # --------------------------------------------------------- param server
    def fetch_model(self):
        """baristanet.py:85-97: GET latest_model, load it, return the iteration."""
        if self.driver is None:
            return self.dummy_fetch_model()
        req = urllib.request.Request("http://%s/api/v1/latest_model" % self.driver,
                                     headers={"Content-Type": "application/deepQ"})
        message = urllib.request.urlopen(req).read()
        self.iteration = messaging.load_model_message(message, self.dqn)
        return self.iteration

    def dummy_fetch_model(self):
        """baristanet.py:99-103 with the 'ii' header the loader expects (the
        reference's dummy path builds an 'i' message, messaging.py:72 vs :91)."""
        message = messaging.create_message(self.dqn.split(self.dqn.get_flat(0), "Q"),
                                           self.iteration)
        return messaging.load_model_message(message, self.dqn)

    def send_gradient_update(self):
        """baristanet.py:105-123: POST the Q gradients; returns the reply body."""
        if self.driver is None:
            return self.dummy_send_gradient_update()
        message = messaging.create_gradient_message(self.dqn)
        req = urllib.request.Request("http://%s/api/v1/update_model" % self.driver,
                                     headers={"Content-Type": "application/deepQ"},
                                     data=message)
        return urllib.request.urlopen(req).read()

    def dummy_send_gradient_update(self):
        messaging.create_gradient_message(self.dqn)
        return b"OK" if np.random.rand() < 0.98 else b"ERROR"

    # -------------------------------------------------------------- compute
    def forward(self, end=None):
        if end == "Q_out":
            self.dqn.forward_q()
        else:
            self.dqn.forward_backward()

    def full_pass(self):
        """baristanet.py:138-140: forward + backward on the bound minibatch."""
        return self.dqn.forward_backward()

    def select_action(self, state, batch_size=1):
        """baristanet.py:142-146: argmax_a Q(s, a) (first max).  ``state`` is
        one (4,S,S) stack or a batch; only the n given states are evaluated."""
        s = np.asarray(state)
        n = 1 if s.ndim == 3 else s.shape[0]
        a = self.dqn.select_action(s.reshape(n, 4, self.dqn.frame, self.dqn.frame))
        return int(a[0]) if (batch_size == 1 and n == 1) else a[:max(batch_size, n)]

    def log(self):
        """Monitoring hook of the reference (NetLogger); a no-op here."""
