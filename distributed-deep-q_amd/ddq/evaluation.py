"""Snapshots and policy evaluation -- host drivers over the
GPU network.

* ``save_snapshot(snapshot_name, model)``: tasks.py:25-34 (``saveSnapshot``):
  pickles ``dict(model)`` ({name: [W, b]}) to ``snapshot_name + str(now)``.
  The reference also mirrors it into a Redis dict; here the files are the
  store.  ``ParamServer(on_snapshot=save_snapshot)`` reproduces the
  server's every-``snapshot_freq``-iterations hook (server.py:74-77).
* ``load_snapshot(path)``: reads such a file with an unpickler that only
  admits numpy arrays and builtin containers (no code runs from the file).
* ``PolicyEvaluator(architecture_file, model_file).evaluate(model,
  num_trials)``: evaluation.py:10-51 -- batch_size Snake engines play
  greedily in lock step, one batched ``select_action`` (the GPU Q tower,
  ``ddq_select_action``) per move; a finished game adds its score and the
  engine restarts, until ``num_trials`` games are done; returns the average
  score.  ``max_moves`` (default None = the reference's unbounded games) ends
  a game that has not finished after that many moves, for drivers that
  cannot risk a policy that circles forever.
* ``evaluate_model(barista_net, model, num_batches)``: q_convergence.py:15-25
  -- mean of Q_out over ``num_batches`` minibatches sampled from the net's
  dataset.
* ``start(architecture_file, model_file, snapshots, ...)``: evaluation.py:
  54-72 over snapshot files instead of Redis keys; returns {name: average}.
"""
from __future__ import annotations

import glob
import os
import pickle
import random
from datetime import datetime

import numpy as np

from .expgain import ExpGain, generate_preprocessor
from .snake import SnakeGame, gray_scale


def save_snapshot(snapshot_name, model, directory="."):
    """tasks.py:25-34.  Returns the file written."""
    filename = os.path.join(directory, snapshot_name + str(datetime.now()))
    snap = {k: [np.array(a, np.float32) for a in v] for k, v in dict(model).items()}
    with open(filename, "wb") as f:
        pickle.dump(snap, f, protocol=2)
    return filename


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("_codecs", "encode"),
        ("builtins", "dict"), ("builtins", "list"), ("collections", "OrderedDict"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError("snapshot refers to %s.%s: not loaded" % (module, name))


def load_snapshot(path):
    """{name: [W, b]} from a snapshot file (numpy arrays and containers only)."""
    with open(path, "rb") as f:
        snap = _SafeUnpickler(f, encoding="latin1").load()
    if not isinstance(snap, dict):
        raise ValueError("%s: not a snapshot dict" % path)
    return {k: [np.asarray(a, np.float32) for a in v] for k, v in snap.items()}


class PolicyEvaluator:
    """evaluation.py:10-51."""

    def __init__(self, architecture_file, model_file, net=None, seed=None, max_moves=None):
        from .barista.baristanet import BaristaNet
        self.net = net if net is not None else BaristaNet(architecture_file, model_file, None)
        self.batch_size = self.net.batch_size
        self.max_moves = max_moves
        game = SnakeGame(random.Random(seed))
        preprocessor = generate_preprocessor(self.net.state.shape[2:], gray_scale)
        self.engines = [ExpGain(self.net, ["w", "a", "s", "d"], preprocessor, game.cpu_play,
                                None, game.encode_state())
                        for _ in range(self.batch_size)]

    def evaluate(self, model, num_trials):
        """Runs ``num_trials`` games and returns the average score."""
        from .barista.netutils import set_net_params
        if model is not None:
            set_net_params(self.net, model)
        for eg in self.engines:
            eg.reset_game()
        total_score = 0
        trials_completed = 0
        scores = [0] * self.batch_size
        moves = [0] * self.batch_size
        while trials_completed < num_trials:
            states = np.stack([eg.get_preprocessed_state() for eg in self.engines])
            actions = self.net.select_action(states, batch_size=self.batch_size)
            for i, (action, eg) in enumerate(zip(actions, self.engines)):
                scores[i] += eg.play_action(eg.actions[int(action)])
                moves[i] += 1
                if eg.game_over or (self.max_moves is not None and moves[i] >= self.max_moves):
                    total_score += scores[i]
                    trials_completed += 1
                    if trials_completed == num_trials:
                        break
                    eg.reset_game()
                    scores[i] = 0
                    moves[i] = 0
        return float(total_score) / num_trials


def evaluate_model(barista_net, model, num_batches):
    """q_convergence.py:15-25: average Q_out over ``num_batches`` minibatches."""
    from .barista.netutils import set_net_params
    if model is not None:
        set_net_params(barista_net, model)
    avg_q = 0.0
    for _ in range(num_batches):
        barista_net.load_minibatch()
        barista_net.forward(end="Q_out")
        avg_q += float(np.mean(barista_net.blobs["Q_out"].data))
    return avg_q / num_batches


def start(architecture_file, model_file, snapshots="centralModel-*", num_trials=32,
          results=None, recompute=False, evaluator=None):
    """evaluation.py:54-72 over snapshot files (a glob or a list) instead of
    Redis keys.  ``results`` (a dict) carries earlier averages; entries are
    recomputed only with ``recompute``."""
    results = {} if results is None else results
    paths = sorted(glob.glob(snapshots)) if isinstance(snapshots, str) else list(snapshots)
    pe = evaluator
    for path in paths:
        key = os.path.basename(path)
        if key in results and not recompute:
            continue
        if pe is None:
            pe = PolicyEvaluator(architecture_file, model_file)
        results[key] = pe.evaluate(load_snapshot(path), num_trials)
    return results
