"""Minimal HDF5 reader/writer for the replay dataset file (host side).

The reference keeps its replay ring in an HDF5 file through h5py
(replay.py:23-68 create/reopen, :185-192 persist on ``__del__``): four
datasets in the root group -- ``state`` u8 (N,4,S,S), ``action`` u8 (N,),
``reward`` i16 (N,), ``non_terminal`` bool (N,) -- and two scalar attributes
``head`` / ``valid`` on ``state``.  h5py is not importable in this image's
Python, so this module reads and writes exactly that layout with no
dependency beyond numpy:

* ``write_replay`` emits the file h5py itself writes by default (superblock
  version 0, a symbol-table root group -- v1 B-tree, SNOD node, local heap --
  version-1 object headers, contiguous layout, h5py's bool enum
  ``{FALSE: 0, TRUE: 1}`` over int8), with the data blocks 4 KiB aligned so
  the state block can be filled in place through a memory map (a 1M-slot
  64x64 ring is 16.4 GB);
* ``read_replay`` / ``H5File`` read files written by h5py (and so by the
  reference): superblock 0-3, symbol-table or compact link groups,
  version-1/2 object headers with continuation blocks, contiguous or compact
  data (an unallocated dataset reads as zeros, the default fill), integer,
  float and bool-enum types, scalar or simple attributes.  Chunked or
  filtered storage and dense (fractal-heap) groups are rejected with an
  error naming the feature.

Tests: ``tests/test_h5.py`` reads a file the reference's own ``replay.py``
wrote (fixture from ``oracle/gen_hdf5_golden.py``) and, where
/opt/conda/bin/python3.9 has h5py, has h5py read what this writer wrote.
"""
from __future__ import annotations

import os
import struct

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF

REPLAY_NAMES = ("state", "action", "reward", "non_terminal")


class H5Error(ValueError):
    pass


def _pad8(n):
    return (n + 7) & ~7


# ---------------------------------------------------------------------------
# reader
# ---------------------------------------------------------------------------

class Dataset:
    def __init__(self, f, name, shape, dtype, addr, size, compact, attrs):
        self._f, self.name, self.shape, self.dtype = f, name, tuple(shape), dtype
        self.addr, self.size, self.compact, self.attrs = addr, size, compact, attrs

    def read(self, mmap=False):
        n = int(np.prod(self.shape, dtype=np.int64))
        if self.compact is not None:
            return np.frombuffer(self.compact, self.dtype, n).reshape(self.shape).copy()
        if self.addr == UNDEF or n == 0:        # never written: the default fill (0)
            return np.zeros(self.shape, self.dtype)
        if self.size < n * self.dtype.itemsize:
            raise H5Error("dataset %s: storage %d B < %d B" % (self.name, self.size,
                                                              n * self.dtype.itemsize))
        off = self._f.base + self.addr
        if mmap:
            return np.memmap(self._f.path, self.dtype, "r", off, self.shape)
        with open(self._f.path, "rb") as fp:
            fp.seek(off)
            a = np.fromfile(fp, self.dtype, n)
        if a.size != n:
            raise H5Error("dataset %s: file truncated" % self.name)
        return a.reshape(self.shape)


class H5File:
    """Root-group datasets of an HDF5 file (read only)."""

    def __init__(self, path):
        self.path = path
        with open(path, "rb") as fp:
            self.buf = memoryview(fp.read(1 << 20))
            fp.seek(0, 2)
            self.flen = fp.tell()
        self._fp = open(path, "rb")
        try:
            self._superblock()
            self.datasets = {}
            for name, oh in self._group(self.root):
                msgs = self._ohdr(oh)
                if any(t == 0x08 for t, _ in msgs):
                    self.datasets[name] = self._dataset(name, msgs)
        finally:
            self._fp.close()

    # -- raw access -----------------------------------------------------------
    def _rd(self, addr, n):
        a = self.base + addr
        if a + n <= len(self.buf):
            return bytes(self.buf[a:a + n])
        if a + n > self.flen:
            raise H5Error("read past end of file at %d" % a)
        self._fp.seek(a)
        return self._fp.read(n)

    def _o(self, b, p):   # offset-sized field
        return int.from_bytes(b[p:p + self.so], "little"), p + self.so

    def _l(self, b, p):   # length-sized field
        return int.from_bytes(b[p:p + self.sl], "little"), p + self.sl

    # -- superblock ------------------------------------------------------------
    def _superblock(self):
        pos = 0
        while pos < self.flen and bytes(self.buf[pos:pos + 8]) != SIGNATURE:
            pos = 512 if pos == 0 else pos * 2
        if pos >= self.flen:
            raise H5Error("%s: not an HDF5 file" % self.path)
        b = bytes(self.buf[pos:pos + 256])
        ver = b[8]
        if ver in (0, 1):
            self.so, self.sl = b[13], b[14]
            p = 24 if ver == 0 else 28
            self.base = 0
            base, p = int.from_bytes(b[p:p + self.so], "little"), p + self.so
            p += 3 * self.so                          # free space, eof, driver
            p += self.so                              # root entry: link name offset
            self.root, p = int.from_bytes(b[p:p + self.so], "little"), p + self.so
            self.base = base if base != UNDEF else pos
        elif ver in (2, 3):
            self.so, self.sl = b[9], b[10]
            p = 12
            base = int.from_bytes(b[p:p + self.so], "little")
            p += 3 * self.so                          # base, extension, eof
            self.root = int.from_bytes(b[p:p + self.so], "little")
            self.base = base
        else:
            raise H5Error("superblock version %d not supported" % ver)

    # -- object headers ----------------------------------------------------------
    def _ohdr(self, addr):
        head = self._rd(addr, 16)
        msgs = []
        if head[:4] == b"OHDR":
            ver, flags = head[4], head[5]
            if ver != 2:
                raise H5Error("object header v2 signature with version %d" % ver)
            p = 6 + (16 if flags & 0x20 else 0) + (4 if flags & 0x10 else 0)
            w = 1 << (flags & 3)
            h = self._rd(addr, p + w)
            size = int.from_bytes(h[p:p + w], "little")
            blocks = [(addr + p + w, size)]       # messages + gap (checksum follows)
            tracked = bool(flags & 0x04)
            while blocks:
                a, n = blocks.pop(0)
                b = self._rd(a, n)
                q = 0
                while q + 4 <= n:
                    t = b[q]
                    sz = int.from_bytes(b[q + 1:q + 3], "little")
                    mf = b[q + 3]
                    q += 4 + (2 if tracked else 0)
                    if q + sz > n:
                        break
                    data = b[q:q + sz]
                    q += sz
                    if mf & 0x02:
                        raise H5Error("shared object header messages not supported")
                    if t == 0x10:
                        ca, cl = int.from_bytes(data[:self.so], "little"), \
                            int.from_bytes(data[self.so:self.so + self.sl], "little")
                        if self._rd(ca, 4) != b"OCHK":
                            raise H5Error("bad continuation block")
                        blocks.append((ca + 4, cl - 8))
                    else:
                        msgs.append((t, data))
            return msgs
        ver, nmsg = head[0], int.from_bytes(head[2:4], "little")
        if ver != 1:
            raise H5Error("object header version %d not supported" % ver)
        size = int.from_bytes(head[8:12], "little")
        blocks = [(addr + 16, size)]
        while blocks and len(msgs) < nmsg:
            a, n = blocks.pop(0)
            b = self._rd(a, n)
            q = 0
            while q + 8 <= n and len(msgs) < nmsg:
                t = int.from_bytes(b[q:q + 2], "little")
                sz = int.from_bytes(b[q + 2:q + 4], "little")
                mf = b[q + 4]
                data = b[q + 8:q + 8 + sz]
                q += 8 + sz
                if mf & 0x02:
                    raise H5Error("shared object header messages not supported")
                if t == 0x10:
                    ca, cl = int.from_bytes(data[:self.so], "little"), \
                        int.from_bytes(data[self.so:self.so + self.sl], "little")
                    blocks.append((ca, cl))
                msgs.append((t, data))
        return msgs

    # -- groups ------------------------------------------------------------------
    def _group(self, addr):
        msgs = self._ohdr(addr)
        out = []
        for t, d in msgs:
            if t == 0x11:                         # symbol table: v1 B-tree + local heap
                bt, p = self._o(d, 0)
                hp, _ = self._o(d, p)
                heap = self._heap(hp)
                for name_off, oh in self._btree(bt):
                    out.append((heap[name_off:heap.index(b"\0", name_off)].decode(), oh))
            elif t == 0x06:                       # link message (compact group)
                out.extend(self._link(d))
            elif t == 0x02:                       # link info: dense storage?
                fh = int.from_bytes(d[2 + (8 if d[1] & 1 else 0):][:self.so], "little")
                if fh != UNDEF:
                    raise H5Error("dense (fractal heap) groups not supported")
        return out

    def _heap(self, addr):
        h = self._rd(addr, 8 + 2 * self.sl + self.so)
        if h[:4] != b"HEAP":
            raise H5Error("bad local heap")
        size, p = self._l(h, 8)
        _, p = self._l(h, p)
        da, _ = self._o(h, p)
        return self._rd(da, size)

    def _btree(self, addr):
        h = self._rd(addr, 8 + 2 * self.so)
        if h[:4] != b"TREE" or h[4] != 0:
            raise H5Error("bad group B-tree node")
        level, used = h[5], int.from_bytes(h[6:8], "little")
        body = self._rd(addr + 8 + 2 * self.so, used * (self.sl + self.so) + self.sl)
        out = []
        for i in range(used):
            p = i * (self.sl + self.so) + self.sl
            child, _ = self._o(body, p)
            if level > 0:
                out.extend(self._btree(child))
            else:
                out.extend(self._snod(child))
        return out

    def _snod(self, addr):
        h = self._rd(addr, 8)
        if h[:4] != b"SNOD":
            raise H5Error("bad symbol table node")
        n = int.from_bytes(h[6:8], "little")
        ent = 2 * self.so + 24
        b = self._rd(addr + 8, n * ent)
        return [(int.from_bytes(b[i * ent:i * ent + self.so], "little"),
                 int.from_bytes(b[i * ent + self.so:i * ent + 2 * self.so], "little"))
                for i in range(n)]

    def _link(self, d):
        flags = d[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = d[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        w = 1 << (flags & 3)
        n = int.from_bytes(d[p:p + w], "little")
        p += w
        name = d[p:p + n].decode()
        p += n
        if ltype != 0:
            return []                              # soft / external links: not datasets here
        return [(name, int.from_bytes(d[p:p + self.so], "little"))]

    # -- datasets ------------------------------------------------------------------
    def _dataspace(self, d):
        ver, rank, flags = d[0], d[1], d[2]
        p = 8 if ver == 1 else 4
        if ver == 2 and d[3] == 2:
            return None                            # null dataspace
        return tuple(int.from_bytes(d[p + i * self.sl:p + (i + 1) * self.sl], "little")
                     for i in range(rank))

    def _dtype(self, d):
        cls, ver = d[0] & 0x0F, d[0] >> 4
        bits = d[1] | (d[2] << 8) | (d[3] << 16)
        size = int.from_bytes(d[4:8], "little")
        order = ">" if bits & 1 else "<"
        if cls == 0:                               # fixed point
            return np.dtype("%s%s%d" % (order, "i" if bits & 0x08 else "u", size)), 12
        if cls == 1:                               # IEEE float
            return np.dtype("%sf%d" % (order, size)), 20
        if cls == 8:                               # enumeration
            nmem = bits & 0xFFFF
            base, bl = self._dtype(d[8:])
            p = 8 + bl
            names = []
            for _ in range(nmem):
                e = d.index(b"\0", p)
                names.append(d[p:e].decode())
                p = p + _pad8(e - p + 1) if ver < 3 else e + 1
            vals = np.frombuffer(d[p:p + nmem * base.itemsize], base)
            p += nmem * base.itemsize
            mem = dict(zip(names, vals.tolist()))
            if base.itemsize == 1 and mem == {"FALSE": 0, "TRUE": 1}:
                return np.dtype(bool), p           # h5py's bool
            return base, p
        raise H5Error("datatype class %d not supported" % cls)

    def _layout(self, d):
        ver = d[0]
        if ver in (3, 4):                          # v4: same compact / contiguous form
            cls = d[1]
            if cls == 0:
                n = int.from_bytes(d[2:4], "little")
                return UNDEF, n, bytes(d[4:4 + n])
            if cls == 1:
                a, p = self._o(d, 2)
                s, _ = self._l(d, p)
                return a, s, None
            raise H5Error("chunked / virtual dataset layout not supported")
        if ver in (1, 2):
            rank, cls = d[1], d[2]
            if cls != 1:
                raise H5Error("layout v%d class %d not supported" % (ver, cls))
            a, p = self._o(d, 8)
            dims = [int.from_bytes(d[p + 4 * i:p + 4 * i + 4], "little") for i in range(rank)]
            return a, int(np.prod(dims, dtype=np.int64)), None
        raise H5Error("layout message version %d not supported" % ver)

    def _attr(self, d):
        ver = d[0]
        nlen = int.from_bytes(d[2:4], "little")
        tlen = int.from_bytes(d[4:6], "little")
        slen = int.from_bytes(d[6:8], "little")
        p = 8
        if ver == 3:
            p += 1
        pad = _pad8 if ver == 1 else (lambda n: n)
        name = d[p:p + nlen].split(b"\0")[0].decode()
        p += pad(nlen)
        dt, _ = self._dtype(d[p:p + tlen])
        p += pad(tlen)
        shape = self._dataspace(d[p:p + slen])
        p += pad(slen)
        n = int(np.prod(shape, dtype=np.int64)) if shape else 1
        val = np.frombuffer(d[p:p + n * dt.itemsize], dt, n)
        return name, (val.reshape(shape) if shape else val[0])

    def _dataset(self, name, msgs):
        shape = dt = lay = None
        attrs = {}
        for t, d in msgs:
            if t == 0x01:
                shape = self._dataspace(d)
            elif t == 0x03:
                dt, _ = self._dtype(d)
            elif t == 0x08:
                lay = self._layout(d)
            elif t == 0x0B:
                raise H5Error("dataset %s: filtered storage not supported" % name)
            elif t == 0x0C:
                k, v = self._attr(d)
                attrs[k] = v
        if shape is None or dt is None or lay is None:
            raise H5Error("dataset %s: incomplete object header" % name)
        return Dataset(self, name, shape, dt, lay[0], lay[1], lay[2], attrs)


def read_replay(path, mmap_state=False):
    """Replay file -> dict(state, action, reward, non_terminal, head, valid),
    or None if the file lacks any of the four datasets (the reference then
    creates them, replay.py:29, :47-62)."""
    f = H5File(path)
    if not all(n in f.datasets for n in REPLAY_NAMES):
        return None
    st = f.datasets["state"]
    if len(st.shape) != 4:
        raise H5Error("state dataset must be 4-D (N,4,S,S), got %s" % (st.shape,))
    N = st.shape[0]
    out = {"state": st.read(mmap=mmap_state).astype(np.uint8, copy=False)}
    for n, dt in (("action", np.uint8), ("reward", np.int16), ("non_terminal", bool)):
        a = f.datasets[n].read()
        if a.shape != (N,):
            raise H5Error("%s dataset shape %s != (%d,)" % (n, a.shape, N))
        out[n] = a.astype(dt, copy=False)
    out["head"] = int(st.attrs.get("head", 0))
    out["valid"] = int(st.attrs.get("valid", 0))
    return out


# ---------------------------------------------------------------------------
# writer (the layout h5py writes for the reference's file)
# ---------------------------------------------------------------------------

def _dt_int(size, signed):
    return struct.pack("<BBBBIHH", 0x10, 0x08 if signed else 0, 0, 0, size, 0, 8 * size)


_DT = {
    "u1": _dt_int(1, False),
    "i2": _dt_int(2, True),
    "i8": _dt_int(8, True),
    # h5py bool: enum {FALSE: 0, TRUE: 1} over signed int8
    "b1": struct.pack("<BBBBI", 0x18, 2, 0, 0, 1) + _dt_int(1, True)
          + b"FALSE\0\0\0" + b"TRUE\0\0\0\0" + b"\x00\x01",
}


def _msg(t, data, flags=0):
    data = data + b"\0" * (_pad8(len(data)) - len(data))
    return struct.pack("<HHB3x", t, len(data), flags) + data


def _ohdr(msgs):
    body = b"".join(msgs)
    return struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body)) + body


def _dataspace(shape):
    return struct.pack("<BBBB4x", 1, len(shape), 1 if shape else 0, 0) + \
        b"".join(struct.pack("<Q", s) for s in shape) * (2 if shape else 0)


def _attr_i64(name, value):
    nm = name.encode() + b"\0"
    dt, ds = _DT["i8"], _dataspace(())
    pad = lambda b: b + b"\0" * (_pad8(len(b)) - len(b))   # noqa: E731
    return struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds)) + pad(nm) + pad(dt) + \
        pad(ds) + struct.pack("<q", int(value))


def write_replay(path, state, action=None, reward=None, non_terminal=None, head=0, valid=0,
                 shape=None):
    """Write the reference's replay file.  ``state`` is an (N,4,S,S) u8 array,
    or -- for large rings, no second host copy -- a callable given the memory
    map of the file's state block (``shape``) that fills it and returns
    ``(action, reward, non_terminal)``."""
    if callable(state):
        if shape is None:
            raise H5Error("shape is required when state is a fill callable")
        shape = tuple(int(x) for x in shape)
    else:
        shape = tuple(state.shape)
    N = shape[0]
    names = sorted(REPLAY_NAMES)                   # SNOD / B-tree order
    # local heap data: "" at 0, names 8-aligned, then one free block (h5py-style)
    heap = b"\0" * 8
    name_off = {}
    for n in names:
        name_off[n] = len(heap)
        e = n.encode() + b"\0"
        heap += e + b"\0" * (_pad8(len(e)) - len(e))
    free_off = len(heap)
    heap += struct.pack("<QQ", 1, 16)              # next free = none (1), size 16
    # fixed-size structures
    SB, ROOT = 0, 96
    root = _ohdr([_msg(0x11, struct.pack("<QQ", 0, 0))])   # patched below
    BT = ROOT + len(root)
    BT_SIZE = 24 + 33 * 8 + 32 * 8                 # group internal K = 16
    HP = BT + BT_SIZE
    HPD = HP + 32
    SN = HPD + len(heap)
    SN_SIZE = 8 + 8 * 40                           # group leaf K = 4
    pos = SN + SN_SIZE
    sizes = {"state": int(np.prod(shape, dtype=np.int64)), "action": N, "reward": 2 * N,
             "non_terminal": N}
    dtypes = {"state": _DT["u1"], "action": _DT["u1"], "reward": _DT["i2"],
              "non_terminal": _DT["b1"]}
    dims = {"state": shape, "action": (N,), "reward": (N,), "non_terminal": (N,)}
    fill = _msg(0x05, bytes([2, 2, 2, 1, 0, 0, 0, 0]))

    def header(n, addr):
        msgs = [_msg(0x01, _dataspace(dims[n])), _msg(0x03, dtypes[n], flags=1), fill,
                _msg(0x08, struct.pack("<BBQQ", 3, 1, addr, sizes[n]))]
        if n == "state":
            msgs += [_msg(0x0C, _attr_i64("head", head)), _msg(0x0C, _attr_i64("valid", valid))]
        return _ohdr(msgs)

    oh_addr, hdrs = {}, {}
    for n in names:                                # header sizes do not depend on addr
        oh_addr[n] = pos
        pos += len(header(n, 0))
    data_addr = {}
    for n in names:
        pos = (pos + 4095) & ~4095
        data_addr[n] = pos
        pos += sizes[n]
    eof = pos
    for n in names:
        hdrs[n] = header(n, data_addr[n])

    sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0) + \
        struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF) + \
        struct.pack("<QQII", 0, ROOT, 1, 0) + struct.pack("<QQ", BT, HP)
    root = _ohdr([_msg(0x11, struct.pack("<QQ", BT, HP))])
    last = names[-1]
    bt = b"TREE" + bytes([0, 0]) + struct.pack("<HQQ", 1, UNDEF, UNDEF) + \
        struct.pack("<QQQ", 0, SN, name_off[last])
    bt += b"\0" * (BT_SIZE - len(bt))
    hp = b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap), free_off, HPD)
    sn = b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names))
    for n in names:
        sn += struct.pack("<QQII16x", name_off[n], oh_addr[n], 0, 0)
    sn += b"\0" * (SN_SIZE - len(sn))
    meta = bytearray(data_addr[names[0]])
    for a, b in ((SB, sb), (ROOT, root), (BT, bt), (HP, hp), (HPD, heap), (SN, sn)):
        meta[a:a + len(b)] = b
    for n in names:
        meta[oh_addr[n]:oh_addr[n] + len(hdrs[n])] = hdrs[n]

    tmp = path + ".tmp%d" % os.getpid()
    try:
        with open(tmp, "wb") as fp:
            fp.truncate(eof)
        if sizes["state"]:
            mm = np.memmap(tmp, np.uint8, "r+", data_addr["state"], shape)
            if callable(state):
                action, reward, non_terminal = state(mm)
            else:
                mm[...] = state
            mm.flush()
            del mm
        arrays = {"action": np.ascontiguousarray(action, np.uint8),
                  "reward": np.ascontiguousarray(reward, "<i2"),
                  "non_terminal": np.ascontiguousarray(non_terminal, bool)}
        for k, a in arrays.items():
            if a.shape != (N,):
                raise H5Error("%s must have shape (%d,), got %s" % (k, N, a.shape))
        with open(tmp, "r+b") as fp:
            fp.write(meta)
            for n in names:
                if n != "state":
                    fp.seek(data_addr[n])
                    fp.write(arrays[n].tobytes())
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
