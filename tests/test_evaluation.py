"""F4 host logic: snapshots (tasks.py:25-34) and the policy evaluator
(evaluation.py:10-72), run on the CPU with the float64 oracle standing in for
the network's action selection (the GPU path is in test_gpu_host.py)."""
import os
import pickle

import numpy as np
import pytest

from ddq import evaluation
from oracle import ref_numpy as ref


class OracleNet:
    """Just what PolicyEvaluator touches: batch_size, state, select_action."""

    def __init__(self, S=16, B=8, seed=3):
        self.batch_size = B
        self.state = np.zeros((B, 4, S, S), np.float32)
        self.pQ = ref.init_params(S, seed=seed)
        self.calls = 0

    def select_action(self, states, batch_size=1):
        self.calls += 1
        return ref.select_action(np.asarray(states, np.float32), self.pQ)


def test_snapshot_round_trip(tmp_path):
    p = ref.init_params(16, seed=1)
    f = evaluation.save_snapshot("centralModel-000500", p, str(tmp_path))
    assert os.path.basename(f).startswith("centralModel-000500")
    got = evaluation.load_snapshot(f)
    assert list(got) == list(p)
    for k in p:
        for a, b in zip(got[k], p[k]):
            np.testing.assert_array_equal(a, np.asarray(b, np.float32))


def test_snapshot_loader_runs_nothing(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    f = tmp_path / "centralModel-000001"
    f.write_bytes(pickle.dumps({"Qconv1": [Evil()]}))
    with pytest.raises(pickle.UnpicklingError):
        evaluation.load_snapshot(str(f))


def test_policy_evaluator_is_deterministic_and_counts_trials():
    net = OracleNet()
    a = evaluation.PolicyEvaluator(None, None, net=net, seed=5, max_moves=200).evaluate(None, 12)
    b = evaluation.PolicyEvaluator(None, None, net=OracleNet(), seed=5,
                                   max_moves=200).evaluate(None, 12)
    assert a == b
    # every game scores at least -1 (one game over) and moves are batched
    assert a >= -1.0 and net.calls >= 12 // net.batch_size


def test_start_over_snapshot_files(tmp_path):
    for it in (500, 1000):
        evaluation.save_snapshot("centralModel-%06d" % it, ref.init_params(16, seed=it),
                                 str(tmp_path))

    class Fake:
        def __init__(self):
            self.seen = []

        def evaluate(self, model, num_trials):
            self.seen.append(float(model["Q_out"][0].sum()))
            return float(len(self.seen))
    fk = Fake()
    res = evaluation.start(None, None, str(tmp_path / "centralModel-*"), num_trials=4,
                           evaluator=fk)
    assert sorted(res.values()) == [1.0, 2.0] and len(fk.seen) == 2
    # already evaluated -> skipped unless recompute
    evaluation.start(None, None, str(tmp_path / "centralModel-*"), results=res, evaluator=fk)
    assert len(fk.seen) == 2
    evaluation.start(None, None, str(tmp_path / "centralModel-*"), results=res,
                     recompute=True, evaluator=fk)
    assert len(fk.seen) == 4
