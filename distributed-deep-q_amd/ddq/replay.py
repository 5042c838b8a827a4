"""HBM-resident experience replay with the interface of replay.py (reference).

``ReplayDataset(filename, state_shape, dset_size=1000, overwrite=False)`` keeps
the ring (u8 (N,4,S,S) states, u8 actions, i16 rewards, bool non_terminal,
head, valid -- replay.py:48-68) in GPU memory; ``add_experience`` and
``sample_direct`` keep the reference semantics (replay.py:70-92, :144-183):

* the index draw is the reference's: ``random.sample`` of distinct indices in
  [0, valid), redrawn while it contains head-1, sorted (host side, Python
  ``random`` -- seedable exactly like the reference);
* the gather runs on the GPU (``ddq_replay_sample``): s <- S[idx],
  s' <- S[idx+1] with only the last row wrapping N-1 -> 0, one-hot action,
  reward and non_terminal of idx+1; bit-exact against the reference.

When the dataset is attached to a ``BaristaNet`` (``net.add_dataset``) the
ring moves into that net's GPU context and ``sample_direct`` on the net's own
minibatch arrays gathers straight into the network's device input (no host
round trip), which is what the reference's zero-copy MEMORY_DATA binding did.
Persistence (replay.py:23-45 reopen, :185-192 persist on ``__del__``):
``save()`` / ``close()`` / ``__del__`` write ``filename`` as the reference's
HDF5 file (``ddq.h5lite``: same datasets, dtypes and head/valid attributes,
readable by h5py and by the reference itself), the state block exported
straight into a memory map of the file; a non-overwrite open of an existing
file -- one the reference wrote, or one written here -- resumes from it,
keeping the file's size with the reference's warning.  A file holding none of
the four datasets is replaced, as the reference creates them.  (An ``.npz``
written by earlier versions of this package is still read.)
"""
from __future__ import annotations

import os
import random

import numpy as np

from . import h5lite
from .net import DeepQNet


class ReplayDataset:
    def __init__(self, filename, state_shape, dset_size=1000, overwrite=False, batch_size=32,
                 device=0, net=None, mode="gpu"):
        self.filename = filename
        self.state_shape = tuple(int(x) for x in state_shape)
        if len(self.state_shape) != 3 or self.state_shape[0] != 4 or \
                self.state_shape[1] != self.state_shape[2]:
            raise ValueError("state_shape must be (4, S, S), got %s" % (self.state_shape,))
        loaded = None
        if filename and not overwrite and os.path.exists(filename):
            loaded = _load_ring(filename)
        if loaded is not None:
            if loaded["state"].shape[1:] != self.state_shape:
                raise ValueError("%s holds states of shape %s, not %s"
                                 % (filename, loaded["state"].shape[1:], self.state_shape))
            if loaded["state"].shape[0] != dset_size:
                print("Warning: dataset loaded from %s is of size %d, not %d as requested. "
                      "Using existing size." % (filename, loaded["state"].shape[0], dset_size))
            dset_size = loaded["state"].shape[0]
        self.dset_size = int(dset_size)
        self._net = net if net is not None else DeepQNet(batch=batch_size,
                                                         frame=self.state_shape[1],
                                                         device=device, mode=mode)
        self._own_net = net is None
        self._net.replay_create(self.dset_size)
        if loaded is not None:
            self._net.replay_import(loaded["state"], loaded["action"], loaded["reward"],
                                    loaded["non_terminal"].astype(np.uint8),
                                    int(loaded["head"]), int(loaded["valid"]))

    # -- reference attributes (replay.py:63-68) --------------------------------
    @property
    def head(self):
        return self._net.replay_info()[0]

    @property
    def valid(self):
        return self._net.replay_info()[1]

    # -- binding to a network context ---------------------------------------
    def attach(self, net):
        """Move the ring into ``net``'s GPU context (one device copy)."""
        if net is self._net:
            return
        st, ac, rw, nt = self._net.replay_export()
        head, valid, _ = self._net.replay_info()
        net.replay_create(self.dset_size)
        net.replay_import(st, ac, rw, nt.astype(np.uint8), head, valid)
        if self._own_net:
            self._net.close()
        self._net, self._own_net = net, False

    # -- replay.py API ------------------------------------------------------
    def add_experience(self, action, reward, state):
        """replay.py:70-92 (state None = terminal; the slot stays stale)."""
        self._net.replay_add(int(action), int(reward), state)

    def draw_indices(self, sample_size):
        """replay.py:147-159: the reference's index draw, on Python ``random``."""
        head, valid, _ = self._net.replay_info()
        if sample_size >= valid:
            raise ValueError("Can't draw sample of size %d from replay dataset of size %d"
                             % (sample_size, valid))
        idx = random.sample(range(0, valid), sample_size)
        while (head - 1) in idx:
            idx = random.sample(range(0, valid), sample_size)
        idx.sort()
        return idx

    def sample_direct(self, state, action, reward, next_state, non_terminal, sample_size):
        """replay.py:144-183.  Gathers on the GPU; the caller's arrays are
        filled unless they are the bound network's own input buffers."""
        idx = self.draw_indices(sample_size)
        if sample_size != self._net.batch:
            st, ac, rw, ns, nt = self._gather_any(np.asarray(idx, np.int32))
        else:
            self._net.replay_sample(np.asarray(idx, np.int32))
            if getattr(state, "_ddq_device_bound", False):
                return
            st, ac, rw, ns, nt = self._net.read_minibatch()
        state[...] = st.reshape(state.shape)
        next_state[...] = ns.reshape(next_state.shape)
        if action.ndim > 1 and action.shape[1] > 1:
            action[...] = ac.reshape(action.shape)
        else:
            action[...] = np.argmax(ac.reshape(len(idx), -1), axis=1).reshape(action.shape)
        reward.flat[:] = rw.ravel()
        non_terminal.flat[:] = nt.ravel()

    def _gather_any(self, idx):
        """Any sample size (the reference gathers into caller arrays of any
        length, replay.py:167-183): the Caffe-layout batch gather
        (ddq_replay_gather_batch_async) into device buffers, then to the host."""
        import torch
        n = int(idx.size)
        bufs = self._net.batch_buffers(n)
        bufs["idx"].copy_(torch.from_numpy(idx))
        torch.cuda.current_stream(bufs["idx"].device).synchronize()   # before the ctx stream reads
        self._net.replay_gather_batch(bufs)                          # checks (and syncs) the ctx
        return tuple(bufs[k].cpu().numpy() for k in ("state", "action", "reward", "next_state",
                                                      "non_terminal"))

    def sample(self, sample_size):
        """Tuple form (the reference's ``sample`` is broken, replay.py:135-136;
        this returns what it evidently intended)."""
        S = self.state_shape[1]
        st = np.empty((sample_size, 4, S, S), np.float32)
        ns = np.empty_like(st)
        ac = np.empty((sample_size, 4, 1, 1), np.float32)
        rw = np.empty((sample_size, 1, 1, 1), np.float32)
        nt = np.empty((sample_size, 1, 1, 1), np.float32)
        self.sample_direct(st, ac, rw, ns, nt, sample_size)
        return st, ac, rw, ns, nt

    def save(self):
        """Persist the ring as the reference's HDF5 file (replay.py:185-192)."""
        if not self.filename:
            return
        head, valid, cap = self._net.replay_info()
        S = self.state_shape[1]
        # states: device -> memory map of the file's state block, one copy
        h5lite.write_replay(self.filename, lambda mm: self._net.replay_export(state_out=mm)[1:],
                            head=head, valid=valid, shape=(cap, 4, S, S))

    def close(self):
        if getattr(self, "_net", None) is not None and self._net.ctx:
            try:
                self.save()
            finally:
                if self._own_net:
                    self._net.close()
        self._net = None

    def __del__(self):   # replay.py:185-192 persists on destruction
        try:
            self.close()
        except Exception:
            pass


def _load_ring(filename):
    """The reference's HDF5 replay file (or a legacy npz) -> ring dict, or None
    when the file holds no replay datasets."""
    with open(filename, "rb") as fp:
        magic = fp.read(8)
    if magic[:2] == b"PK":
        with np.load(filename, allow_pickle=False) as f:
            return {k: f[k] for k in f.files}
    return h5lite.read_replay(filename, mmap_state=True)
