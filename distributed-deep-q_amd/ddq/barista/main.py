"""Barista worker server (main.py, reference): a TCP loop on 127.0.0.1:port
where one request byte 'G' triggers one training step (main.py:37-112):
fetch the model from the param server, generate one experience (ε-greedy
acting through the GPU Q tower), sample a minibatch from the HBM replay, run
the forward/backward pass on the GPU, push the Q gradients, reply.

    python -m ddq.barista.main <train_val.prototxt> <model.npz|none>
        [--port 50001] [--driver 127.0.0.1:5500|None] [--dataset replay-dataset.hdf5]
        [--dset-size 1000] [--overwrite] [--debug] [--initial-replay 20000]

``--mode gpu`` (default) runs libddq_hip.so; ``--mode cpu`` runs the same
step on the host through the CPU twin libddq_cpu.so (main.py:128,149-151, the
reference's Caffe CPU mode: BASELINE configs[0]).
"""
from __future__ import annotations

import argparse
import os
import socket
import time

from .. import expgain as eg
from ..replay import ReplayDataset
from ..snake import SnakeGame, gray_scale
from . import GRAD_UPDATE, DARWIN_UPDATE, MSG_LENGTH, netutils
from .baristanet import BaristaNet


def recv_all(sock, size):
    message = b""
    while len(message) < size:
        chunk = sock.recv(4096)
        if not chunk:
            break
        message += chunk
    return message


def process_connection(sock, net, exp_gain, debug=False):
    """main.py:37-58 / :61-112 (the non-debug handler's NameError at :46 is
    not reproduced; both modes run the same step)."""
    message = recv_all(sock, MSG_LENGTH)
    if message == GRAD_UPDATE:
        iteration_num = net.fetch_model()
        exp_gain.generate_experience(iteration_num)
        net.load_minibatch()
        tic = time.time()
        net.full_pass()
        toc = time.time()
        if debug:
            print("    * step took % 0.2f milliseconds." % (1000 * (toc - tic)))
            print("Loss:", netutils.extract_net_data(net, ("loss",))["loss"])
        response = net.send_gradient_update()
        net.log()
        sock.sendall(response if isinstance(response, bytes) else str(response).encode())
    elif message == DARWIN_UPDATE:
        raise NotImplementedError("Darwinian SGD not implemented")
    else:
        print("Unknown request:", message)
    sock.close()


def issue_ready_signal(idx):
    """main.py:115-120: flags/__BARISTA_READY__.<port>."""
    os.makedirs("flags", exist_ok=True)
    open("flags/__BARISTA_READY__.%d" % idx, "w").close()


def get_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("architecture")
    ap.add_argument("model")
    ap.add_argument("--solver", default=None)
    ap.add_argument("--mode", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--port", type=int, default=50001)
    ap.add_argument("--driver", default="127.0.0.1:5500")
    ap.add_argument("--dataset", default="replay-dataset.hdf5")   # main.py:131
    ap.add_argument("--dset-size", dest="dset_size", type=int, default=1000)
    ap.add_argument("--overwrite", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--initial-replay", type=int, default=20000)
    ap.add_argument("--max-requests", type=int, default=0, help="exit after N requests (tests)")
    args = ap.parse_args(argv)
    if args.driver == "None":
        args.driver = None
    return args


def build_worker(args):
    model = None if args.model in ("none", "None") else args.model
    net = BaristaNet(args.architecture, model, args.driver, logpath=None, mode=args.mode)
    replay = ReplayDataset(args.dataset, net.state[0].shape, dset_size=args.dset_size,
                           overwrite=args.overwrite, batch_size=net.batch_size, mode=args.mode)
    net.add_dataset(replay)
    game = SnakeGame()
    pre = eg.generate_preprocessor(net.state.shape[2:], gray_scale)
    exp_gain = eg.ExpGain(net, ["w", "a", "s", "d"], pre, game.cpu_play, replay,
                          game.encode_state())
    if args.overwrite:                                  # main.py:176-178
        for _ in range(min(args.initial_replay, args.dset_size)):
            exp_gain.generate_experience(0)
    return net, replay, exp_gain


def main(argv=None):
    args = get_args(argv)
    net, replay, exp_gain = build_worker(args)
    server = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    server.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    server.bind(("127.0.0.1", args.port))
    server.listen(5)
    print("* Starting BARISTA server: listening on port %d." % args.port, flush=True)
    issue_ready_signal(args.port)
    served = 0
    try:
        while args.max_requests == 0 or served < args.max_requests:
            client, _ = server.accept()
            process_connection(client, net, exp_gain, args.debug)
            served += 1
    finally:
        server.close()
        replay.close()


if __name__ == "__main__":
    main()
