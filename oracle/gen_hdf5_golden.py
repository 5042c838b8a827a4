"""ORACLE fixture generator -- test infrastructure only.

Pins the replay file format with the REFERENCE's own
``replay.py`` (read in place from /root/reference, never copied), run under
/opt/conda/bin/python3.9 (h5py 3.3.0):

    /opt/conda/bin/python3.9 oracle/gen_hdf5_golden.py tests/golden

* ``h5_ref_s16.hdf5`` + ``h5_ref_s16.npz``: a file the reference
  wrote (create, 15 writes into a 12-slot ring incl. terminals, persist on
  ``__del__``, replay.py:23-92, :185-192) and the ring contents it held.
* ``h5_resume_in.hdf5``: the file ``ddq.h5lite.write_replay`` makes from
  the arrays in ``h5_resume.npz`` (``in_*``); the reference reopens it
  (overwrite=False, replay.py:29-45), and the fixture records what it read
  (``read_*``), then 3 more writes and a ``sample_direct`` with a scripted
  index draw (``idx``, ``out_*``), and the file it persisted
  (``h5_resume_out.hdf5``, final ring in ``fin_*``).

The shipped build never runs this file; the GPU box never sees /root/reference.
"""
import builtins
import os
import random
import shutil
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True   # never write into the read-only reference tree
builtins.xrange = range           # replay.py is Python-2 source (xrange)
sys.path.insert(0, REF)
sys.path.insert(1, os.path.join(HERE, "..", "distributed-deep-q_amd", "ddq"))
import replay as ref_replay       # noqa: E402  (the reference module itself)
import h5lite                     # noqa: E402  (the build's writer, pure numpy)

S = 16


def ring(ds):
    return dict(state=np.asarray(ds.state[...]), action=ds.action.copy(),
                reward=ds.reward.copy(), non_terminal=ds.non_terminal.copy(),
                head=int(ds.head), valid=int(ds.valid))


def writes(rng, n, p_term=0.25):
    out = []
    for _ in range(n):
        st = None if rng.random() < p_term else rng.integers(0, 256, (4, S, S)).astype(np.uint8)
        out.append((int(rng.integers(0, 4)), int(rng.integers(-3, 4)), st))
    return out


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    rng = np.random.default_rng(77)
    with tempfile.TemporaryDirectory() as td:
        # -- A: a file written by the reference --------------------------------
        fa = os.path.join(td, "a.hdf5")
        ds = ref_replay.ReplayDataset(fa, (4, S, S), dset_size=12, overwrite=True)
        for a, r, st in writes(rng, 15):
            ds.add_experience(a, r, st)
        exp = ring(ds)
        del ds                                    # reference __del__ persists + closes
        shutil.copy(fa, os.path.join(outdir, "h5_ref_s16.hdf5"))
        np.savez_compressed(os.path.join(outdir, "h5_ref_s16.npz"), **exp)

        # -- B: the reference resumes from a file the build wrote -------------
        N = 10
        inp = dict(state=rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8),
                   action=rng.integers(0, 4, N).astype(np.uint8),
                   reward=rng.integers(-2, 3, N).astype(np.int16),
                   non_terminal=rng.random(N) < 0.7, head=7, valid=N)
        fb = os.path.join(td, "b.hdf5")
        h5lite.write_replay(fb, inp["state"], inp["action"], inp["reward"],
                            inp["non_terminal"], inp["head"], inp["valid"])
        shutil.copy(fb, os.path.join(outdir, "h5_resume_in.hdf5"))
        ds = ref_replay.ReplayDataset(fb, (4, S, S), dset_size=N, overwrite=False)
        read = ring(ds)
        for a, r, st in writes(rng, 3, p_term=0.34):
            ds.add_experience(a, r, st)
        B = 5
        script = [[9, 0, 4, 2, 7]]                # N-1 drawn: its s' wraps to slot 0
        orig = random.sample
        ref_replay.random.sample = lambda pop, k: list(script.pop(0)) if script else orig(pop, k)
        o = dict(state=np.zeros((B, 4, S, S), np.float32), next_state=np.zeros((B, 4, S, S), np.float32),
                 action=np.zeros((B, 4, 1, 1), np.float32), reward=np.zeros((B, 1, 1, 1), np.float32),
                 non_terminal=np.zeros((B, 1, 1, 1), np.float32))
        ds.sample_direct(o["state"], o["action"], o["reward"], o["next_state"],
                         o["non_terminal"], B)
        ref_replay.random.sample = orig
        fin = ring(ds)
        del ds
        shutil.copy(fb, os.path.join(outdir, "h5_resume_out.hdf5"))
        rec = {}
        for pre, d in (("in_", inp), ("read_", read), ("fin_", fin), ("out_", o)):
            rec.update({pre + k: np.asarray(v) for k, v in d.items()})
        rec["idx"] = np.asarray(sorted([9, 0, 4, 2, 7]), np.int64)
        np.savez_compressed(os.path.join(outdir, "h5_resume.npz"), **rec)
        print("ref file: head=%d valid=%d; resume: read head=%d valid=%d, final head=%d valid=%d"
              % (exp["head"], exp["valid"], read["head"], read["valid"], fin["head"], fin["valid"]))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "tests/golden")
