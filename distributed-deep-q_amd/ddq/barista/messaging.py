"""Wire format between a Barista worker and the parameter server, compatible with
barista/messaging.py (reference) -- framing and fp32 payload byte-identical, the
header an equivalent pickle (see below):

* model message (server -> worker, messaging.py:13-40):
    struct.pack('ii', iteration, hlen) + header + raw fp32 blobs
* gradient / net message (worker -> server, messaging.py:43-79):
    struct.pack('i', hlen) + header + raw fp32 blobs of the ``Q*`` params only
* header: pickle (protocol 2, the protocol Python 2 ``cPickle.dumps(.., -1)``
  writes) of an OrderedDict {param name: [blob shape, ...]} in parameter order.
  Python 2 cPickle decodes it to the same OrderedDict, but the bytes are not
  cPickle's own (BINUNICODE names against SHORT_BINSTRING, Python 3's memo
  numbering), so the length prefix (this header's own length) differs too;
  the reference never compares header bytes, it decodes them.  The
  loaders use only element counts (:111-112) or reshape to the header shapes
  (:159-161).

``params`` arguments are mappings name -> [W, b] of numpy arrays (the shape
``caffe.Net.params`` exposes through ``.data``/``.diff``) or a ``BaristaNet`` /
``DeepQNet``, whose blobs are read from / written to the GPU in one flat copy.
"""
from __future__ import annotations

import collections
import pickle
import struct
import zlib

import numpy as np

from . import DTYPE, DTYPE_SIZE


def _pack(meta_items, arrays, compress):
    meta = collections.OrderedDict(meta_items)
    header = pickle.dumps(meta, 2)
    data = b"".join(np.ascontiguousarray(a, DTYPE).tobytes() for a in arrays)
    if compress:
        data = zlib.compress(data)
    return header, data


def create_message(params, iteration_num, compress=False):
    """messaging.py:13-40 (model message; every param in dict order)."""
    items, arrays = [], []
    for name in params:
        blobs = params[name]
        items.append((name, [tuple(np.shape(b)) for b in blobs]))
        for b in blobs:
            if np.asarray(b).dtype != DTYPE:
                raise AssertionError("parameter %s is not float32" % name)
            arrays.append(b)
    header, data = _pack(items, arrays, compress)
    return struct.pack("ii", int(iteration_num), len(header)) + header + data


def create_net_message(params, attr="diff", compress=False):
    """messaging.py:43-73: only parameters whose name starts with 'Q'."""
    items, arrays = [], []
    for name in params:
        if name[0] != "Q":
            continue
        blobs = [getattr(b, attr) if hasattr(b, attr) else b for b in params[name]]
        items.append((name, [tuple(np.shape(b)) for b in blobs]))
        arrays.extend(blobs)
    header, data = _pack(items, arrays, compress)
    return struct.pack("i", len(header)) + header + data


def _net_params(net, attr):
    """Q-tower {name: [W, b]} of a BaristaNet/DeepQNet, one device copy."""
    dq = getattr(net, "dqn", net)
    flat = dq.get_grads_flat() if attr == "diff" else dq.get_flat(0)
    return dq.split(flat, "Q")


def create_gradient_message(net, compress=False):
    """messaging.py:76-79."""
    return create_net_message(_net_params(net, "diff"), "diff", compress)


def create_model_message(net, compress=False):
    """messaging.py:82-83."""
    return create_net_message(_net_params(net, "data"), "data", compress)


class _HeaderUnpickler(pickle.Unpickler):
    """Headers arrive from the network: resolve no global except OrderedDict
    (lists, tuples, strings and ints need none).  A reference header (Python 2
    cPickle protocol 2) decodes unchanged; anything else -- a pickle that would
    call a function or build another class -- is refused instead of run."""

    def find_class(self, module, name):
        if (module, name) in (("collections", "OrderedDict"), ("builtins", "list"),
                              ("builtins", "tuple")):
            return super().find_class(module, name)
        raise pickle.UnpicklingError("message header refers to %s.%s: refused" % (module, name))


def _load_header(raw):
    import io
    header = _HeaderUnpickler(io.BytesIO(raw), encoding="latin1").load()
    if not isinstance(header, dict):
        raise ValueError("message header is not a mapping")
    for name, shapes in header.items():
        if not isinstance(name, str) or not isinstance(shapes, (list, tuple)) or not all(
                isinstance(sh, (list, tuple)) and all(isinstance(d, int) and d >= 0 for d in sh)
                for sh in shapes):
            raise ValueError("malformed message header entry %r" % (name,))
    return header


def _parse(message, with_iteration, compressed):
    if with_iteration:
        iteration_num, hlen = struct.unpack("ii", message[:8])
        off = 8
    else:
        iteration_num, (hlen,) = None, struct.unpack("i", message[:4])
        off = 4
    header = _load_header(message[off:off + hlen])
    data = message[off + hlen:]
    if compressed:
        data = zlib.decompress(data)
    return iteration_num, header, data


def load_net_message(message, net, attr="data", compressed=False):
    """messaging.py:87-119: assign every header blob into ``net`` by element
    count (KeyError for an unknown name).  Returns the iteration number."""
    iteration_num, header, data = _parse(message, True, compressed)
    dq = getattr(net, "dqn", net)
    known = set(dq.q_names) | set(dq.p_names)
    arrays = collections.OrderedDict()
    idx = 0
    for name in header:
        if name not in known:
            raise KeyError("Received parameter %s not in model's architecture." % name)
        arrays[name] = []
        for shape in header[name]:
            n = int(np.prod(shape)) * DTYPE_SIZE
            arrays[name].append(np.frombuffer(data[idx:idx + n], DTYPE))
            idx += n
    if attr == "data":
        _partial_set(dq, arrays)
    else:
        grads = dq.split(dq.get_grads_flat(), "Q")
        for name, blobs in arrays.items():
            for g, b in zip(grads[name], blobs):
                g.flat[:] = b
        dq.set_grads_flat(dq.join(grads, "Q"))
    return iteration_num


def _partial_set(dq, arrays):
    for which, prefix in ((0, "Q"), (1, "P")):
        names = [prefix + k[1:] for k in dq.q_names]
        if not any(n in arrays for n in names):
            continue
        cur = dq.split(dq.get_flat(which), prefix)
        for n in names:
            if n in arrays:
                for dst, src in zip(cur[n], arrays[n]):
                    dst.flat[:] = src
        dq.set_flat(which, dq.join(cur, prefix))


def load_model_message(message, net):
    """messaging.py:121-125."""
    return load_net_message(message, net, "data")


def load_gradient_message(message, compressed=False):
    """messaging.py:128-164: {name: [ndarray (read-only, header shape), ...]}."""
    _, header, data = _parse(message, False, compressed)
    grads, idx = {}, 0
    for name in header:
        grads[name] = []
        for shape in header[name]:
            n = int(np.prod(shape)) * DTYPE_SIZE
            grads[name].append(np.frombuffer(data[idx:idx + n], DTYPE).reshape(shape))
            idx += n
    return grads


def load_model_params(message, compressed=False):
    """Decode a model message into (iteration, {name: [ndarray]}) without a net."""
    it, header, data = _parse(message, True, compressed)
    out, idx = collections.OrderedDict(), 0
    for name in header:
        out[name] = []
        for shape in header[name]:
            n = int(np.prod(shape)) * DTYPE_SIZE
            out[name].append(np.frombuffer(data[idx:idx + n], DTYPE).reshape(shape))
            idx += n
    return it, out
