"""Multi-GPU data parallelism: one process per GPU.

Each rank owns a full theta_Q/theta_P replica, its own HBM replay shard and its
own device index stream (seed = base + rank).  Per step the flat gradient is
summed over ranks with one RCCL all-reduce inside the step graph
(``ddq_allreduce_grads``), then every rank applies the same update -- the
reference's "W gradients pushed to the parameter server" with the HTTP/Redis
round trip (baristanet.py:105-123, server.py:196-209) replaced by xGMI.

``torch.distributed`` (gloo) is used only to bootstrap: broadcast rank 0's
128-byte RCCL unique id, barriers, and max-over-ranks timing.
"""
from __future__ import annotations

import os
import time


def env_ranks():
    """(rank, world_size, local_rank) from torchrun-style environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_process_group(rank, world, backend="gloo"):
    import torch.distributed as dist
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        dist.init_process_group(backend, rank=rank, world_size=world)
    return dist


def broadcast_unique_id(rank, make_uid):
    """Rank 0 creates the communicator id, every rank receives the same bytes."""
    import torch.distributed as dist
    obj = [make_uid() if rank == 0 else None]
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast_object_list(obj, src=0)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise RuntimeError("bad communicator id")
    return bytes(uid)


def setup_comm(net, rank, world):
    """Create the RCCL communicator of ``net`` (a DeepQNet) over all ranks."""
    from .net import DeepQNet
    uid = broadcast_unique_id(rank, DeepQNet.comm_unique_id)
    net.comm_init(uid, world, rank)
    return uid


def index_seed(base, rank):
    """Per-rank device index stream (PCG64(1234 + rank))."""
    return int(base) + int(rank)


def max_over_ranks(value):
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok):
    """True only if ``ok`` holds on every rank (gloo MIN all-reduce): a
    fallback decision every rank takes together, so no rank proceeds into a
    collective the others have abandoned."""
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def choose_step_mode(net, cfg, modes, log=None):
    """Prepare (capture + instantiate, nothing launched) the first step mode
    of ``modes`` -- (name, overlap) pairs, name in "pipelined" / "graph" /
    "eager" -- that succeeds on EVERY rank; the decision is collective.
    Returns the chosen (name, overlap)."""
    from ._lib import DDQError
    for name, overlap in modes:
        cfg.overlap = int(bool(overlap))
        ok = True
        try:
            net.step_prepare(cfg, name)
        except DDQError as e:
            ok = False
            if log:
                log("step mode %s%s failed to prepare: %s" % (name, "+overlap" if overlap else "", e))
        if all_ranks_ok(ok):
            return name, overlap
    raise RuntimeError("no step mode could be prepared on every rank")


def ticket_store(world, rank=0, prefix="ddq/async"):
    """The key-value store that hands out async tickets: the default process
    group's store (a TCPStore every rank reaches) when one is initialised,
    an in-process HashStore for a single rank."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        from torch.distributed import distributed_c10d as c10d
        return dist.PrefixStore(prefix, c10d._get_default_store())
    if world > 1:
        raise RuntimeError("ticket_store: world > 1 needs an initialised process group")
    return dist.PrefixStore(prefix, dist.HashStore())


class AsyncTicketLoop:
    """Arrival-order pushes of the asynchronous param server over RCCL ranks
    (include/ddq_hip.h DDQ_EXCHANGE_ASYNC, ddq_async_tick).

    The reference's workers push whenever their gradient is ready and the
    one server applies pushes in the order they arrive (main.py:61-112,
    server.py:196-209).  Here a rank whose gradient is ready
    (``net.async_ready()``) takes the next ticket from a shared store (an
    atomic counter: ``store.add``) and publishes ``tk/<t> = rank``; every rank
    executes tick t as soon as its owner is known, in ticket order, so all
    ranks enqueue the same RCCL send / recv sequence.  A fast worker takes
    several tickets while a slow one takes one.  No device ever waits for a
    ticket: the order is decided on the host, the ticks are enqueued
    asynchronously and the gradient of the next tick computes meanwhile.

    Ticket state lives in the loop: a ticket this rank took that lies past the
    end of a ``run`` (it became ready while the last ticks were executed) is
    executed by the next ``run`` of the same loop, on every rank.  Each loop
    instance keys its tickets under an instance number of its own (the n-th
    loop a rank creates on ``store`` is instance n -- every rank creates its
    loops in the same order), so a new loop never replays an older loop's
    tickets; tickets still held when a loop is dropped are dropped with it.
    """

    def __init__(self, net, cfg, store, rank, world):
        import torch.distributed as dist
        self.net, self.cfg = net, cfg
        self.rank, self.world = int(rank), int(world)
        self.instance = store.add("instances/%d" % self.rank, 1) - 1
        self.store = dist.PrefixStore("i%d" % self.instance, store)
        self.next = 0            # next ticket to execute
        self.holding = False     # this rank holds a ticket not yet executed
        self.mine = -1           # ... that ticket's number

    def run(self, npush, poll_s=50e-6, spin_s=2e-3, timeout_s=600.0):
        """Execute the next npush ticks (whoever pushes); returns their workers.

        The loop spins (no sleep) for spin_s after its last progress -- a
        sleep of tens of microseconds lasts several times that and the device
        idles meanwhile -- then polls every poll_s.  The spin polls only local
        state (this worker's gradient readiness, its own ticket); the store
        server is asked about other ranks' tickets at most once per poll_s, so
        W spinning ranks do not flood it.  A ticket this rank takes is its own
        to execute: when it is the next one, no store read is needed (one add
        + one set per own push; other ranks' tickets: one check + one get)."""
        net, store = self.net, self.store
        net.async_begin(self.cfg)
        order = []
        end = self.next + int(npush)
        idle_since = time.perf_counter()
        last_check = -1.0
        while self.next < end:
            progressed = False
            if not self.holding and net.async_ready():
                self.mine = store.add("ticket", 1) - 1
                store.set("tk/%d" % self.mine, str(self.rank))
                self.holding = True
                progressed = True
            w = None
            if self.holding and self.mine == self.next:
                w = self.rank
            else:
                now = time.perf_counter()
                if now - last_check >= poll_s:
                    last_check = now
                    key = "tk/%d" % self.next
                    if store.check([key]):
                        w = int(store.get(key))
            if w is not None:
                net.async_tick(self.cfg, w)
                order.append(w)
                if w == self.rank:
                    self.holding = False
                self.next += 1
                progressed = True
            now = time.perf_counter()
            if progressed:
                idle_since = now
            else:
                if now - idle_since > timeout_s:
                    raise RuntimeError("async ticket loop: no progress for %.0f s" % timeout_s)
                if now - idle_since > spin_s:
                    time.sleep(poll_s)
        return order
