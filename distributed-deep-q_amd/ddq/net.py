"""DeepQNet: the MI355X replacement of the pycaffe ``caffe.Net`` used by the
reference worker (barista/baristanet.py:16, :41-43, :136-146) for the deepq
network of models/deepq/train_val.prototxt.

One DeepQNet owns one ``ddq_ctx`` (one GPU, one HIP stream) holding both
towers (Q and the frozen target P), the minibatch, the optimizer state and,
optionally, the HBM replay ring.  All arithmetic runs in libddq_hip.so.
"""
from __future__ import annotations

import collections
import ctypes

import numpy as np

from . import _lib
from ._lib import check, ptr

GAMMA = 0.85        # models/deepq/train_val.prototxt:473
NUM_ACTIONS = 4     # barista/constants.py:8
NFRAME = 4          # expgain.py:9

BLOBS = {"Q_out": 4, "P_out": 4, "Q_sa": 1, "P_sa": 1, "target_Q_sa": 1, "loss": 0}


class DeepQNet:
    """Device-resident deepq network (both towers) + minibatch + replay ring."""

    def __init__(self, batch=32, frame=16, device=0, gamma=GAMMA, mode="gpu"):
        """mode "gpu": libddq_hip.so on HIP device ``device``; "cpu": the CPU
        twin libddq_cpu.so (the reference's Caffe CPU mode, no GPU)."""
        self.mode = mode
        self.lib = _lib.load(mode=mode)
        self.batch, self.frame, self.device = int(batch), int(frame), int(device)
        desc = _lib.NetDesc(self.batch, self.frame, NFRAME, NUM_ACTIONS, gamma)
        ctx = ctypes.c_void_p()
        check(self.lib.ddq_create(ctypes.byref(ctx), self.device, ctypes.byref(desc)), None, self.lib)
        self.ctx = ctx
        self.num_params = int(self.lib.ddq_num_params(ctx))
        n = _lib._i32()
        arr = (_lib.BlobDesc * 10)()
        self._check(self.lib.ddq_param_layout(ctx, arr, 10, ctypes.byref(n)))
        # pycaffe net.params order: Q tower then P tower (train_val.prototxt order)
        self.layout = collections.OrderedDict()
        for d in arr[: n.value]:
            name = d.name.decode()
            self.layout.setdefault(name, []).append(
                (tuple(int(x) for x in d.shape), int(d.offset), int(d.count)))
        self.q_names = list(self.layout)
        self.p_names = ["P" + k[1:] for k in self.q_names]
        self.has_replay = False

    # ------------------------------------------------------------------ utils
    def _check(self, rc):
        return check(rc, self.ctx, self.lib)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ddq_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        self._check(self.lib.ddq_synchronize(self.ctx))

    def inject_fault(self, fault="meet_timeout"):
        """Arm a failpoint (tests): "meet_timeout" -- the next eager step's fc4
        chain launches one workgroup short (ddq_inject_fault); None disarms."""
        f = _lib.FAULT_NONE if fault is None else {"meet_timeout": _lib.FAULT_MEET_TIMEOUT}[fault]
        self._check(self.lib.ddq_inject_fault(self.ctx, f))

    def small_path(self):
        """(on, reason off): the four-launch small-map step (S = 16) or not."""
        buf = ctypes.create_string_buffer(256)
        on = self.lib.ddq_small_path(self.ctx, buf, 256)
        if on < 0:
            self._check(on)
        return bool(on), buf.value.decode()

    # ------------------------------------------------------------- parameters
    def stream(self):
        """The ctx's HIP stream handle (int), e.g. for torch.cuda.ExternalStream."""
        h = ctypes.c_void_p()
        self._check(self.lib.ddq_get_stream(self.ctx, ctypes.byref(h)))
        return int(h.value or 0)

    def set_flat(self, which, flat):
        flat = np.ascontiguousarray(flat, np.float32).ravel()
        self._check(self.lib.ddq_set_params(self.ctx, which, ptr(flat), flat.size, 0))

    def get_flat(self, which):
        out = np.empty(self.num_params, np.float32)
        self._check(self.lib.ddq_get_params(self.ctx, which, ptr(out), out.size, 0))
        return out

    def get_grads_flat(self):
        out = np.empty(self.num_params, np.float32)
        self._check(self.lib.ddq_get_grads(self.ctx, ptr(out), out.size, 0))
        return out

    def set_grads_flat(self, flat):
        flat = np.ascontiguousarray(flat, np.float32).ravel()
        self._check(self.lib.ddq_set_grads(self.ctx, ptr(flat), flat.size, 0))

    def split(self, flat, prefix="Q"):
        """flat tower buffer -> OrderedDict{name: [W, b]} with Caffe 4-D shapes."""
        out = collections.OrderedDict()
        for qname, blobs in self.layout.items():
            name = prefix + qname[1:]
            out[name] = [flat[o:o + c].reshape(s) for (s, o, c) in blobs]
        return out

    def join(self, params, prefix="Q"):
        flat = np.empty(self.num_params, np.float32)
        for qname, blobs in self.layout.items():
            name = prefix + qname[1:]
            for (s, o, c), arr in zip(blobs, params[name]):
                a = np.asarray(arr, np.float32)
                if a.size != c:
                    raise ValueError("param %s: %d elements, expected %d" % (name, a.size, c))
                flat[o:o + c] = a.ravel()
        return flat

    def set_params(self, params):
        """Assign Q* and/or P* blobs from a {name: [W, b]} mapping."""
        for which, prefix in ((0, "Q"), (1, "P")):
            if all((prefix + k[1:]) in params for k in self.q_names):
                self.set_flat(which, self.join(params, prefix))

    def get_params(self, include_p=True):
        out = self.split(self.get_flat(0), "Q")
        if include_p:
            out.update(self.split(self.get_flat(1), "P"))
        return out

    def sync_target(self):
        """special_update_transform_model (param-server/server.py:127-137)."""
        self._check(self.lib.ddq_sync_target(self.ctx))

    # -------------------------------------------------------------- minibatch
    def write_minibatch(self, state=None, action=None, reward=None, next_state=None,
                        non_terminal=None):
        B, S = self.batch, self.frame

        def prep(a, shape):
            if a is None:
                return None
            a = np.ascontiguousarray(a, np.float32)
            if a.size != int(np.prod(shape)):
                raise ValueError("minibatch array has %d elements, expected shape %s"
                                 % (a.size, shape))
            return a

        st = prep(state, (B, NFRAME, S, S))
        ns = prep(next_state, (B, NFRAME, S, S))
        ac = prep(action, (B, NUM_ACTIONS))
        rw = prep(reward, (B,))
        nt = prep(non_terminal, (B,))
        self._check(self.lib.ddq_write_minibatch(self.ctx, ptr(st), ptr(ac), ptr(rw), ptr(ns),
                                                 ptr(nt)))

    def read_minibatch(self):
        B, S = self.batch, self.frame
        st = np.empty((B, NFRAME, S, S), np.float32)
        ns = np.empty((B, NFRAME, S, S), np.float32)
        ac = np.empty((B, NUM_ACTIONS, 1, 1), np.float32)
        rw = np.empty((B, 1, 1, 1), np.float32)
        nt = np.empty((B, 1, 1, 1), np.float32)
        self._check(self.lib.ddq_read_minibatch(self.ctx, ptr(st), ptr(ac), ptr(rw), ptr(ns),
                                                ptr(nt)))
        return st, ac, rw, ns, nt

    # ----------------------------------------------------------------- compute
    def forward_backward(self):
        """net.forward(); net.backward()  (baristanet.py:138-140).  Returns loss."""
        loss = ctypes.c_float()
        self._check(self.lib.ddq_forward_backward(self.ctx, ctypes.byref(loss)))
        return float(loss.value)

    def forward_q(self):
        """net.forward(end='Q_out') on the bound minibatch."""
        self._check(self.lib.ddq_forward_q(self.ctx))

    def blob(self, name):
        if name not in BLOBS:
            raise KeyError(name)
        B = self.batch
        n = B * BLOBS[name] if BLOBS[name] else 1
        out = np.empty(n, np.float32)
        self._check(self.lib.ddq_read_blob(self.ctx, name.encode(), ptr(out), n))
        if name in ("Q_out", "P_out"):
            return out.reshape(B, 4, 1, 1)
        if name == "loss":
            return out.reshape(())
        return out.reshape(B, 1, 1, 1)

    def pool_mask(self, layer):
        """Q-tower pool routing bytes (B,C,H,W) of the last forward_backward."""
        C = 32 if layer == 1 else 64
        hp = self.frame >> layer
        out = np.empty((self.batch, C, hp, hp), np.uint8)
        self._check(self.lib.ddq_read_pool_mask(self.ctx, int(layer), ptr(out), out.size))
        return out

    def select_action(self, states_u8):
        """argmax_a Q(s, a) for n stacked uint8 states (n,4,S,S)."""
        s = np.ascontiguousarray(states_u8)
        if s.dtype != np.uint8:
            s = np.clip(np.rint(s), 0, 255).astype(np.uint8)
        s = s.reshape(-1, NFRAME, self.frame, self.frame)
        out = np.empty(s.shape[0], np.int32)
        self._check(self.lib.ddq_select_action(self.ctx, ptr(s), s.shape[0], ptr(out)))
        return out

    # ------------------------------------------------------------------- apply
    def apply(self, rule="rmsprop", lr=1e-4, decay=0.9, eps=1e-8, momentum=0.9,
              weight_decay=0.0005):
        cfg = _lib.update_cfg(rule, lr, decay, eps, momentum, weight_decay)
        self._check(self.lib.ddq_apply(self.ctx, ctypes.byref(cfg)))

    def reset_optimizer(self):
        self._check(self.lib.ddq_reset_optimizer(self.ctx))

    def optimizer_state(self):
        out = np.empty(self.num_params, np.float32)
        self._check(self.lib.ddq_get_optimizer_state(self.ctx, ptr(out), out.size))
        return out

    # ------------------------------------------------------------------ replay
    def replay_create(self, capacity):
        self._check(self.lib.ddq_replay_create(self.ctx, int(capacity)))
        self.has_replay = True

    def replay_add(self, action, reward, state):
        st = None
        if state is not None:
            st = np.ascontiguousarray(state, np.uint8)
            if st.size != NFRAME * self.frame * self.frame:
                raise ValueError("state must have %d elements" % (NFRAME * self.frame ** 2))
        self._check(self.lib.ddq_replay_add(self.ctx, int(action), int(reward), ptr(st)))

    def replay_info(self):
        h, v, c = _lib._i64(), _lib._i64(), _lib._i64()
        self._check(self.lib.ddq_replay_info(self.ctx, ctypes.byref(h), ctypes.byref(v),
                                             ctypes.byref(c)))
        return int(h.value), int(v.value), int(c.value)

    def replay_import(self, state, action, reward, non_terminal, head, valid):
        st = np.ascontiguousarray(state, np.uint8)
        ac = np.ascontiguousarray(action, np.uint8)
        rw = np.ascontiguousarray(reward, np.int16)
        nt = np.ascontiguousarray(non_terminal, np.uint8)
        self._check(self.lib.ddq_replay_import(self.ctx, ptr(st), ptr(ac), ptr(rw), ptr(nt),
                                               ac.size, int(head), int(valid)))

    def replay_export(self, state_out=None):
        """Ring contents; ``state_out`` (e.g. a memory map of the replay file's
        state block) receives the states in place."""
        _, _, cap = self.replay_info()
        S = self.frame
        if state_out is not None:
            if state_out.shape != (cap, NFRAME, S, S) or state_out.dtype != np.uint8 or \
                    not state_out.flags.c_contiguous:
                raise ValueError("state_out must be a C-contiguous u8 array of shape %s"
                                 % ((cap, NFRAME, S, S),))
            st = state_out
        else:
            st = np.empty((cap, NFRAME, S, S), np.uint8)
        ac = np.empty(cap, np.uint8)
        rw = np.empty(cap, np.int16)
        nt = np.empty(cap, np.uint8)
        self._check(self.lib.ddq_replay_export(self.ctx, ptr(st), ptr(ac), ptr(rw), ptr(nt), cap))
        return st, ac, rw, nt.astype(bool)

    def replay_sample(self, sorted_idx):
        idx = np.ascontiguousarray(sorted_idx, np.int32)
        self._check(self.lib.ddq_replay_sample(self.ctx, ptr(idx), idx.size))

    def replay_sample_device(self, seed):
        self._check(self.lib.ddq_replay_sample_device_async(self.ctx, int(seed)))

    def replay_fill_tiled(self, state, action, reward, non_terminal, head, valid):
        """Tile a pool of transitions over the whole ring on the device."""
        st = np.ascontiguousarray(state, np.uint8)
        ac = np.ascontiguousarray(action, np.uint8)
        rw = np.ascontiguousarray(reward, np.int16)
        nt = np.ascontiguousarray(non_terminal, np.uint8)
        self._check(self.lib.ddq_replay_fill_tiled(self.ctx, ptr(st), ptr(ac), ptr(rw), ptr(nt),
                                                   ac.size, int(head), int(valid)))

    def batch_buffers(self, n):
        """Device (torch) output buffers for replay_sample_batch (Caffe shapes)."""
        import torch
        dev = torch.device("cuda", self.device)
        S = self.frame
        f = dict(dtype=torch.float32, device=dev)
        return {"idx": torch.empty(n, dtype=torch.int32, device=dev),
                "state": torch.empty((n, NFRAME, S, S), **f),
                "action": torch.empty((n, NUM_ACTIONS, 1, 1), **f),
                "reward": torch.empty((n, 1, 1, 1), **f),
                "next_state": torch.empty((n, NFRAME, S, S), **f),
                "non_terminal": torch.empty((n, 1, 1, 1), **f)}

    def replay_sample_batch(self, bufs, seed, check=True):
        """Large-batch device draw + gather into ``bufs`` (batch_buffers)."""
        n = bufs["idx"].numel()
        p = [bufs[k].data_ptr() for k in ("idx", "state", "action", "reward", "next_state",
                                         "non_terminal")]
        self._check(self.lib.ddq_replay_sample_batch_async(self.ctx, n, int(seed), *p))
        if check:
            self._check(self.lib.ddq_replay_status(self.ctx))

    def replay_gather_batch(self, bufs, check=True):
        """Caffe-layout gather of the sorted indices already in bufs['idx']."""
        n = bufs["idx"].numel()
        p = [bufs[k].data_ptr() for k in ("state", "action", "reward", "next_state",
                                         "non_terminal")]
        self._check(self.lib.ddq_replay_gather_batch_async(self.ctx, bufs["idx"].data_ptr(), n,
                                                           *p))
        if check:
            self._check(self.lib.ddq_replay_status(self.ctx))

    def replay_draws(self):
        """Device index draws made so far (device RNG stream position)."""
        d = _lib._i64()
        self._check(self.lib.ddq_replay_draws(self.ctx, ctypes.byref(d)))
        return int(d.value)

    def index_log_enable(self, draws):
        """Log every device-drawn index set in a ring of ``draws`` entries."""
        self._check(self.lib.ddq_index_log_enable(self.ctx, int(draws)))

    def index_log(self, first, n):
        """(n, B) sorted index sets of device draws first .. first+n-1."""
        out = np.empty((int(n), self.batch), np.int32)
        self._check(self.lib.ddq_index_log_read(self.ctx, int(first), int(n), ptr(out)))
        return out

    def read_indices(self):
        out = np.empty(self.batch, np.int32)
        self._check(self.lib.ddq_read_indices(self.ctx, ptr(out), self.batch))
        return out

    # -------------------------------------------------------------------- step
    def step_cfg(self, rule="rmsprop", lr=1e-4, target_period=10, allreduce=False, seed=0,
                 exchange=None, overlap=False, store_grads=True, **kw):
        """exchange: "none" | "allreduce" | "sharded" | "server" | "async" (include/ddq_hip.h
        enum ddq_exchange); allreduce=True is shorthand for "allreduce".
        store_grads=False: exchange-free steps do not store fc4's weight gradient
        (DDQ_STEP_NO_GRAD_STORE; the update is the same, bit for bit)."""
        if exchange is None:
            exchange = "allreduce" if allreduce else "none"
        ex = _lib.EXCHANGES[exchange] if isinstance(exchange, str) else int(exchange)
        flags = 0 if store_grads else _lib.STEP_NO_GRAD_STORE
        return _lib.StepCfg(_lib.update_cfg(rule, lr, **kw), int(target_period), ex, int(seed),
                            int(bool(overlap)), flags)

    def step(self, cfg):
        self._check(self.lib.ddq_step_async(self.ctx, ctypes.byref(cfg)))

    def step_graph(self, cfg, nsteps):
        self._check(self.lib.ddq_step_graph_async(self.ctx, ctypes.byref(cfg), int(nsteps)))

    def step_prepare(self, cfg, mode="pipelined"):
        """Capture and instantiate the graphs of a step mode ("eager", "graph",
        "pipelined") without launching anything."""
        m = {"eager": 0, "graph": 1, "pipelined": 2}[mode]
        self._check(self.lib.ddq_step_prepare(self.ctx, ctypes.byref(cfg), m))

    def step_pipelined(self, cfg, nsteps):
        """nsteps graph steps with step t+1's sample + gather overlapped with step t."""
        self._check(self.lib.ddq_step_pipelined_async(self.ctx, ctypes.byref(cfg), int(nsteps)))

    def profile_step(self, cfg, cap=32):
        names = ctypes.create_string_buffer(16 * cap)
        us = (ctypes.c_float * cap)()
        n = _lib._i32()
        self._check(self.lib.ddq_profile_step(self.ctx, ctypes.byref(cfg), names, us, cap,
                                              ctypes.byref(n)))
        raw = names.raw
        return [(raw[16 * i:16 * i + 16].split(b"\0")[0].decode(), float(us[i]))
                for i in range(min(n.value, cap))]

    def time_layer(self, name, reps=100):
        """Average device microseconds of one launch of a forward conv layer
        ("conv1_fwd" / "conv2_fwd" / "conv3_fwd"), reps launches back to back."""
        us = ctypes.c_float()
        self._check(self.lib.ddq_time_layer(self.ctx, name.encode(), int(reps), ctypes.byref(us)))
        return float(us.value)

    def step_flops(self):
        return float(self.lib.ddq_step_flops(self.ctx))

    # -------------------------------------------------------------------- comm
    @staticmethod
    def comm_unique_id():
        lib = _lib.load()
        buf = (ctypes.c_uint8 * 128)()
        check(lib.ddq_comm_get_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid, nranks, rank):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.ddq_comm_init(self.ctx, buf, int(nranks), int(rank)))

    @staticmethod
    def group_init(nets):
        """In-process data-parallel group (ddq_group_init): nets[r] is rank r."""
        lib = _lib.load()
        arr = (ctypes.c_void_p * len(nets))(*[n.ctx.value for n in nets])
        check(lib.ddq_group_init(arr, len(nets)))
        return arr

    @staticmethod
    def group_step(nets, cfg, arr=None):
        lib = _lib.load()
        if arr is None:
            arr = (ctypes.c_void_p * len(nets))(*[n.ctx.value for n in nets])
        rc = lib.ddq_group_step(arr, len(nets), ctypes.byref(cfg))
        if rc != 0:
            check(rc, nets[0].ctx)

    @staticmethod
    def group_async_run(nets, cfg, npush, arr=None):
        """Ticket-order async exchange of an in-process group: npush pushes,
        each by the member whose gradient was ready first.  Returns the order."""
        import numpy as np
        lib = _lib.load()
        if arr is None:
            arr = (ctypes.c_void_p * len(nets))(*[n.ctx.value for n in nets])
        order = np.zeros(max(int(npush), 1), np.int32)
        rc = lib.ddq_group_async_run(arr, len(nets), ctypes.byref(cfg), int(npush), ptr(order))
        if rc != 0:
            check(rc, nets[0].ctx)
        return order[:int(npush)]

    @staticmethod
    def group_async_ticks(nets, cfg, order, arr=None):
        """Async ticks of an in-process group in the given worker order."""
        import numpy as np
        lib = _lib.load()
        if arr is None:
            arr = (ctypes.c_void_p * len(nets))(*[n.ctx.value for n in nets])
        o = np.ascontiguousarray(order, np.int32)
        rc = lib.ddq_group_async_ticks(arr, len(nets), ctypes.byref(cfg), int(o.size),
                                       ptr(o) if o.size else None)
        if rc != 0:
            check(rc, nets[0].ctx)

    def async_begin(self, cfg):
        self._check(self.lib.ddq_async_begin(self.ctx, ctypes.byref(cfg)))

    def async_ready(self):
        r = _lib._i32()
        self._check(self.lib.ddq_async_ready(self.ctx, ctypes.byref(r)))
        return bool(r.value)

    def async_tick(self, cfg, worker):
        self._check(self.lib.ddq_async_tick(self.ctx, ctypes.byref(cfg), int(worker)))

    def set_straggle(self, usec):
        """Delay every gradient of this worker by usec (straggler emulation)."""
        self._check(self.lib.ddq_set_straggle(self.ctx, int(usec)))

    def allreduce_grads(self):
        self._check(self.lib.ddq_allreduce_grads(self.ctx))
