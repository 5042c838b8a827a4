"""ctypes binding of libddq_hip.so (include/ddq_hip.h).

There is no fallback: if the HIP library is missing or fails to load, importing
the product path raises.  Build it with ``make -C distributed-deep-q_amd`` (or
``python -c "import __graft_entry__ as g; g.build()"``).

``load(mode="cpu")`` binds libddq_cpu.so instead: the same C-ABI computed on
the host (cpu/twin.cpp), the reference's Caffe CPU mode (main.py --mode cpu).
It is chosen explicitly -- never as a fallback for a missing GPU.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

# DDQ_LIB_PATH: an A/B variant build (tools/ab, `make variant`); the product
# path is the in-tree library
LIB_PATH = os.environ.get("DDQ_LIB_PATH") or \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libddq_hip.so")
CPU_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libddq_cpu.so")
MODES = ("gpu", "cpu")

DDQ_OK, DDQ_EINVAL, DDQ_ENOMEM, DDQ_EHIP, DDQ_ERCCL, DDQ_ESTATE, DDQ_ERANGE = 0, -1, -2, -3, -4, -5, -6
RULES = {"sgd": 0, "rmsprop": 1, "adagrad": 2, "momentum": 3}


class DDQError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("ddq error %d: %s" % (code, msg))
        self.code = code
        self.msg = msg


class NetDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("frame", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("actions", ctypes.c_int32),
                ("gamma", ctypes.c_float)]


class BlobDesc(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 16), ("index", ctypes.c_int32),
                ("shape", ctypes.c_int32 * 4), ("offset", ctypes.c_int64),
                ("count", ctypes.c_int64)]


class UpdateCfg(ctypes.Structure):
    _fields_ = [("rule", ctypes.c_int32), ("lr", ctypes.c_float), ("decay", ctypes.c_float),
                ("eps", ctypes.c_float), ("momentum", ctypes.c_float),
                ("weight_decay", ctypes.c_float)]


class StepCfg(ctypes.Structure):
    _fields_ = [("update", UpdateCfg), ("target_period", ctypes.c_int32),
                ("exchange", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("overlap", ctypes.c_int32), ("flags", ctypes.c_int32)]


STEP_NO_GRAD_STORE = 1     # include/ddq_hip.h DDQ_STEP_NO_GRAD_STORE
FAULT_NONE, FAULT_MEET_TIMEOUT = 0, 1   # include/ddq_hip.h enum ddq_fault

ABI_VERSION = 6
EXCHANGES = {"none": 0, "allreduce": 1, "sharded": 2, "server": 3, "async": 4}


_P = ctypes.c_void_p
_i32, _i64, _u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
_fp = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes)
_SIGS = {
    "ddq_abi_version": (ctypes.c_int, []),
    "ddq_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(NetDesc)]),
    "ddq_destroy": (ctypes.c_int, [_P]),
    "ddq_last_error": (ctypes.c_char_p, [_P]),
    "ddq_set_stream": (ctypes.c_int, [_P, _P]),
    "ddq_synchronize": (ctypes.c_int, [_P]),
    "ddq_inject_fault": (ctypes.c_int, [_P, _i32]),
    "ddq_small_path": (ctypes.c_int, [_P, ctypes.c_char_p, _i32]),
    "ddq_get_stream": (ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    "ddq_num_params": (_i64, [_P]),
    "ddq_param_layout": (ctypes.c_int, [_P, ctypes.POINTER(BlobDesc), _i32, ctypes.POINTER(_i32)]),
    "ddq_set_params": (ctypes.c_int, [_P, _i32, _P, _i64, _i32]),
    "ddq_get_params": (ctypes.c_int, [_P, _i32, _P, _i64, _i32]),
    "ddq_get_grads": (ctypes.c_int, [_P, _P, _i64, _i32]),
    "ddq_set_grads": (ctypes.c_int, [_P, _P, _i64, _i32]),
    "ddq_sync_target": (ctypes.c_int, [_P]),
    "ddq_replay_create": (ctypes.c_int, [_P, _i64]),
    "ddq_replay_add": (ctypes.c_int, [_P, _i32, _i32, _P]),
    "ddq_replay_info": (ctypes.c_int, [_P, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                                       ctypes.POINTER(_i64)]),
    "ddq_replay_import": (ctypes.c_int, [_P, _P, _P, _P, _P, _i64, _i64, _i64]),
    "ddq_replay_export": (ctypes.c_int, [_P, _P, _P, _P, _P, _i64]),
    "ddq_replay_sample": (ctypes.c_int, [_P, _P, _i32]),
    "ddq_replay_sample_device_async": (ctypes.c_int, [_P, _u64]),
    "ddq_read_minibatch": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "ddq_write_minibatch": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "ddq_read_indices": (ctypes.c_int, [_P, _P, _i32]),
    "ddq_replay_fill_tiled": (ctypes.c_int, [_P, _P, _P, _P, _P, _i64, _i64, _i64]),
    "ddq_replay_sample_batch_async": (ctypes.c_int, [_P, _i32, _u64, _P, _P, _P, _P, _P, _P]),
    "ddq_replay_gather_batch_async": (ctypes.c_int, [_P, _P, _i32, _P, _P, _P, _P, _P]),
    "ddq_replay_status": (ctypes.c_int, [_P]),
    "ddq_replay_draws": (ctypes.c_int, [_P, ctypes.POINTER(_i64)]),
    "ddq_index_log_enable": (ctypes.c_int, [_P, _i64]),
    "ddq_index_log_read": (ctypes.c_int, [_P, _i64, _i64, _P]),
    "ddq_forward_backward": (ctypes.c_int, [_P, _fp]),
    "ddq_forward_backward_async": (ctypes.c_int, [_P]),
    "ddq_forward_q": (ctypes.c_int, [_P]),
    "ddq_read_blob": (ctypes.c_int, [_P, ctypes.c_char_p, _P, _i64]),
    "ddq_read_pool_mask": (ctypes.c_int, [_P, _i32, _P, _i64]),
    "ddq_select_action": (ctypes.c_int, [_P, _P, _i32, _P]),
    "ddq_apply": (ctypes.c_int, [_P, ctypes.POINTER(UpdateCfg)]),
    "ddq_apply_async": (ctypes.c_int, [_P, ctypes.POINTER(UpdateCfg)]),
    "ddq_reset_optimizer": (ctypes.c_int, [_P]),
    "ddq_get_optimizer_state": (ctypes.c_int, [_P, _P, _i64]),
    "ddq_comm_get_unique_id": (ctypes.c_int, [_P]),
    "ddq_comm_init": (ctypes.c_int, [_P, _P, _i32, _i32]),
    "ddq_allreduce_grads": (ctypes.c_int, [_P]),
    "ddq_allreduce_grads_async": (ctypes.c_int, [_P]),
    "ddq_step_async": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg)]),
    "ddq_step_graph_async": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg), _i32]),
    "ddq_step_pipelined_async": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg), _i32]),
    "ddq_step_prepare": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg), _i32]),
    "ddq_step_count": (_i64, [_P]),
    "ddq_group_init": (ctypes.c_int, [ctypes.POINTER(_P), _i32]),
    "ddq_group_step": (ctypes.c_int, [ctypes.POINTER(_P), _i32, ctypes.POINTER(StepCfg)]),
    "ddq_group_async_run": (ctypes.c_int, [ctypes.POINTER(_P), _i32, ctypes.POINTER(StepCfg), _i32,
                                           _P]),
    "ddq_group_async_ticks": (ctypes.c_int, [ctypes.POINTER(_P), _i32, ctypes.POINTER(StepCfg),
                                             _i32, _P]),
    "ddq_async_begin": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg)]),
    "ddq_async_ready": (ctypes.c_int, [_P, ctypes.POINTER(_i32)]),
    "ddq_async_tick": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg), _i32]),
    "ddq_set_straggle": (ctypes.c_int, [_P, _i64]),
    "ddq_profile_step": (ctypes.c_int, [_P, ctypes.POINTER(StepCfg), _P, _fp, _i32,
                                        ctypes.POINTER(_i32)]),
    "ddq_time_layer": (ctypes.c_int, [_P, ctypes.c_char_p, _i32, _fp]),
    "ddq_step_flops": (ctypes.c_double, [_P]),
}

EXPORTED = tuple(_SIGS)
_lib = None          # the HIP library (mode "gpu")
_cpu_lib = None      # the CPU twin (mode "cpu")


def load(path=None, mode="gpu"):
    """Load libddq_hip.so (raises if it is absent -- no CPU fallback), or with
    mode="cpu" the CPU twin libddq_cpu.so."""
    global _lib, _cpu_lib
    if mode not in MODES:
        raise ValueError("mode must be one of %s" % (MODES,))
    if mode == "cpu":
        if _cpu_lib is not None:
            return _cpu_lib
        path = path or CPU_LIB_PATH
        if not os.path.exists(path):
            raise ImportError("libddq_cpu.so not found at %s; build it with "
                              "`make -C distributed-deep-q_amd`" % path)
        _cpu_lib = _bind(ctypes.CDLL(path))
        return _cpu_lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise ImportError("libddq_hip.so not found at %s; build it with "
                          "`make -C distributed-deep-q_amd` (hipcc --offload-arch=gfx950)" % path)
    try:  # share torch's HIP runtime when torch is present (same SONAME)
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is plumbing only
        pass
    _lib = _bind(ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL))
    return _lib


def _bind(lib):
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ddq_abi_version() != ABI_VERSION:
        raise ImportError("%s ABI %d != binding ABI %d (rebuild)"
                          % (lib._name, lib.ddq_abi_version(), ABI_VERSION))
    return lib


def check(rc, ctx=None, lib=None):
    if rc != DDQ_OK:
        lib = lib or load()
        msg = lib.ddq_last_error(ctx)
        raise DDQError(rc, msg.decode() if msg else "")
    return rc


def ptr(a):
    """Host pointer of a C-contiguous numpy array (or None)."""
    if a is None:
        return None
    assert isinstance(a, np.ndarray) and a.flags["C_CONTIGUOUS"], "need C-contiguous ndarray"
    return a.ctypes.data_as(ctypes.c_void_p)


def update_cfg(rule="rmsprop", lr=1e-4, decay=0.9, eps=1e-8, momentum=0.9, weight_decay=0.0005):
    """Defaults: param-server/server.py:265-271 (rmsprop, lr 1e-4, decay 0.9),
    eps 1e-8 (server.py:105); momentum/weight_decay: solver.prototxt:9-10."""
    r = RULES[rule] if isinstance(rule, str) else int(rule)
    return UpdateCfg(r, lr, decay, eps, momentum, weight_decay)
