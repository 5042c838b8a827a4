"""GPU, two or more devices: the RCCL exchanges at world size W > 1 against
the in-process group (tests/test_gpu_exchange.py), which runs the same
kernels, shard layout and tick order with the transfers as device copies.

W processes (tests/_rccl_worker.py, rank r on GPU r, one RCCL communicator)
run R steps of an exchange; the parent runs an in-process group of W ctxs on
GPU 0 with the same replay contents, initialisation and cfg.  At W = 2 every
sum has two terms (a + b == b + a in IEEE arithmetic), so every exchange must
agree bit for bit: each rank's Q and P parameters and gradient buffer, and
the optimizer state each owner holds (all of it for the all-reduce).  The
async exchange covers what the world-1 tests cannot: the point-to-point
pushes / pulls and the owner applies on the comm stream while the ctx stream
computes the next gradient.

Skipped on a one-GPU box (RCCL refuses two ranks on one device); named to run
after every other GPU test file.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _rccl_worker as W_  # noqa: E402  (constants and replay contents)


def _ngpu():
    import torch
    return torch.cuda.device_count()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(exchange, world, rounds, tmp_path):
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / ("rank%d.npz" % r))
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_rccl_worker.py"),
                                       exchange, str(rounds), out], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=90)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, "rank %d exit %s:\n%s" % (r, p.returncode, logs[r][-2000:])
    return [np.load(o) for o in outs]


def _group(ddq, exchange, world, rounds):
    from ddq.params import init_params_flat
    theta = init_params_flat(W_.S, seed=42)
    nets = []
    for r in range(world):
        n = ddq.DeepQNet(batch=W_.B, frame=W_.S, device=0)
        n.set_flat(0, theta)
        n.set_flat(1, theta)
        n.replay_create(W_.N)
        n.replay_import(*W_.member_data(r), 0, W_.N)
        nets.append(n)
    arr = ddq.DeepQNet.group_init(nets)
    ex = "async" if exchange == "async-graph" else exchange.replace("-pipelined", "")
    cfg = nets[0].step_cfg("rmsprop", lr=W_.LR, target_period=W_.PERIOD, exchange=ex,
                           seed=W_.SEED)
    for _ in range(rounds):
        ddq.DeepQNet.group_step(nets, cfg, arr)
    res = [dict(q=n.get_flat(0), p=n.get_flat(1), opt=n.optimizer_state(),
                grad=n.get_grads_flat()) for n in nets]
    for n in nets:
        n.close()
    return res


@pytest.mark.skipif("_ngpu() < 2")
@pytest.mark.parametrize("exchange", ["async", "async-graph", "server", "sharded", "allreduce",
                                      "sharded-pipelined", "server-pipelined"])
def test_rccl_two_ranks_equal_in_process_group(exchange, tmp_path):
    import ddq
    world, rounds = 2, 5            # 10 async ticks: special updates at iterations 4 and 8
    ranks = _run_ranks(exchange, world, rounds, tmp_path)
    group = _group(ddq, exchange, world, rounds)
    P = group[0]["q"].size
    L = -(-P // (64 * world)) * 64
    for r in range(world):
        for key in ("q", "p", "grad"):
            np.testing.assert_array_equal(ranks[r][key], group[r][key],
                                          err_msg="%s rank %d %s" % (exchange, r, key))
        sl = slice(0, P) if exchange == "allreduce" else slice(r * L, min((r + 1) * L, P))
        np.testing.assert_array_equal(ranks[r]["opt"][sl], group[r]["opt"][sl],
                                      err_msg="%s rank %d owner optimizer state" % (exchange, r))


@pytest.mark.parametrize("exchange", ["sharded-pipelined", "server-pipelined"])
def test_rccl_worker_world1_pipelined(exchange, tmp_path):
    """The worker's pipelined modes at world size 1 (runs on a one-GPU box):
    the RCCL communicator of one rank, the R steps as one pipelined chain,
    equal to the in-process group of one stepped round by round."""
    import ddq
    world, rounds = 1, 6
    ranks = _run_ranks(exchange, world, rounds, tmp_path)
    group = _group(ddq, exchange, world, rounds)
    for key in ("q", "p", "grad", "opt"):
        np.testing.assert_array_equal(ranks[0][key], group[0][key], err_msg="%s %s" % (exchange, key))
