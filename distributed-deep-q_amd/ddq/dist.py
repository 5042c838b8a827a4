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
