"""One rank of tests/test_gpu_zz_rccl_multi.py: W processes, rank r on GPU r,
an RCCL communicator over all of them (gloo only broadcasts its id), R steps
of one exchange, then the rank's Q / P parameters, optimizer state and last
gradient saved for the parent to compare with an in-process group.

usage: RANK=r WORLD_SIZE=W MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
       python tests/_rccl_worker.py EXCHANGE ROUNDS OUT.npz

EXCHANGE "async-graph": the async exchange stepped as graph replays mixed with
eager rounds (ddq_step_graph_async: one eager round, one K-round graph, then
eager rounds after the replay -- the comm-stream ordering of ADVICE r03).
"sharded-pipelined" / "server-pipelined": that exchange's R steps as one
ddq_step_pipelined_async chain (the next step's draw + gather inside the
shard-apply launch).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-deep-q_amd"))

S, B, N, SEED, PERIOD, LR = 16, 8, 120, 5, 4, 1e-4


def member_data(r):
    """The replay contents of member r (tests/test_gpu_exchange.py make_group)."""
    rng = np.random.default_rng(r)
    return (rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8),
            rng.integers(0, 4, N).astype(np.uint8),
            rng.integers(-1, 2, N).astype(np.int16),
            (rng.random(N) > 0.1).astype(np.uint8))


def main():
    exchange, rounds, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ddq
    from ddq import dist as ddist
    from ddq.params import init_params_flat
    theta = init_params_flat(S, seed=42)
    n = ddq.DeepQNet(batch=B, frame=S, device=rank)
    n.set_flat(0, theta)
    n.set_flat(1, theta)
    n.replay_create(N)
    n.replay_import(*member_data(rank), 0, N)
    ddist.setup_comm(n, rank, world)
    graph = exchange == "async-graph"
    piped = exchange.endswith("-pipelined")
    ex = "async" if graph else exchange.replace("-pipelined", "")
    cfg = n.step_cfg("rmsprop", lr=LR, target_period=PERIOD, exchange=ex, seed=SEED)
    done = 0
    if graph:   # K = PERIOD / gcd(W, PERIOD) rounds per graph, after one eager round
        k = 1 + PERIOD // np.gcd(world, PERIOD)
        n.step_graph(cfg, min(k, rounds))
        done = min(k, rounds)
    if piped:
        n.step_prepare(cfg, "pipelined")
        n.step_pipelined(cfg, rounds)
        done = rounds
    for _ in range(rounds - done):
        n.step(cfg)
    n.synchronize()
    np.savez(out, q=n.get_flat(0), p=n.get_flat(1), opt=n.optimizer_state(),
             grad=n.get_grads_flat())
    dist.barrier()
    n.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
