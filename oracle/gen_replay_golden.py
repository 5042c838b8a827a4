"""ORACLE fixture generator -- test infrastructure only.

Runs the REFERENCE ``replay.py`` (read in place from /root/reference, never
copied) under /opt/conda/bin/python3.9 (the interpreter in this container that
has h5py 3.3.0) and records golden vectors for the minibatch gather
(replay.py:144-183) and the ring write (replay.py:70-92):

    /opt/conda/bin/python3.9 oracle/gen_replay_golden.py tests/golden

Each fixture ``replay_<case>.npz`` holds the reference dataset's storage after
the writes (state u8 (N,4,S,S), action u8, reward i16, non_terminal bool, head,
valid), the sorted index list the reference drew (random.sample is wrapped to
record -- and in the redraw case to script -- its draws; the redraw loop itself
is the reference's), and the five arrays sample_direct wrote.  The shipped
build never runs this file; the GPU box never sees /root/reference.
"""
import builtins
import os
import random
import sys
import tempfile

import numpy as np

REF = "/root/reference"
sys.dont_write_bytecode = True   # never write into the read-only reference tree
builtins.xrange = range           # replay.py is Python-2 source (xrange)
sys.path.insert(0, REF)
import replay as ref_replay       # noqa: E402  (the reference module itself)


class Recorder:
    """Wraps random.sample as seen by replay.py; optionally scripts draws."""

    def __init__(self, script=None):
        self.calls = []
        self.script = list(script or [])
        self._orig = random.sample

    def __call__(self, population, k):
        if self.script:
            out = list(self.script.pop(0))
        else:
            out = self._orig(population, k)
        self.calls.append(list(out))
        return out


def run_case(name, S, N, writes, B, outdir, script=None, seed=0):
    random.seed(seed)
    np.random.seed(seed)
    with tempfile.TemporaryDirectory() as td:
        ds = ref_replay.ReplayDataset(os.path.join(td, "d.hdf5"), (4, S, S),
                                      dset_size=N, overwrite=True)
        for (a, r, st) in writes:
            ds.add_experience(a, r, st)
        rec = Recorder(script)
        ref_replay.random.sample = rec
        state = np.zeros((B, 4, S, S), np.float32)
        next_state = np.zeros((B, 4, S, S), np.float32)
        action = np.zeros((B, 4, 1, 1), np.float32)
        reward = np.zeros((B, 1, 1, 1), np.float32)
        nonterm = np.zeros((B, 1, 1, 1), np.float32)
        err = ""
        try:
            ds.sample_direct(state, action, reward, next_state, nonterm, B)
        except ValueError as e:   # B >= valid
            err = str(e)
        ref_replay.random.sample = rec._orig
        idx = sorted(rec.calls[-1]) if rec.calls else []
        np.savez_compressed(
            os.path.join(outdir, "replay_%s.npz" % name),
            S=S, N=N, B=B, st=np.asarray(ds.state[...]), action=ds.action.copy(),
            reward=ds.reward.copy(), non_terminal=ds.non_terminal.copy(),
            head=int(ds.head), valid=int(ds.valid), idx=np.asarray(idx, np.int64),
            n_draws=len(rec.calls), out_state=state, out_next_state=next_state,
            out_action=action, out_reward=reward, out_non_terminal=nonterm,
            error=np.asarray(err))
        head, valid = int(ds.head), int(ds.valid)
        del ds                    # reference __del__ persists + closes the file
    print(name, "draws=%d" % len(rec.calls), "head=%d valid=%d" % (head, valid),
          "err=%r" % err)


def writes_random(rng, n, S, p_term=0.1):
    out = []
    for _ in range(n):
        a = int(rng.integers(0, 4))
        r = int(rng.integers(-1, 2))
        st = None if rng.random() < p_term else rng.integers(0, 256, (4, S, S)).astype(np.uint8)
        out.append((a, r, st))
    return out


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    rng = np.random.default_rng(2024)
    # plain: partially filled ring, random terminals
    run_case("s16_basic", 16, 64, writes_random(rng, 40, 16), 8, outdir, seed=1)
    # head == 0 after exactly N writes: slot N-1 may be drawn, its s' is slot 0
    w = writes_random(rng, 32, 16)
    run_case("s16_head0_wrap", 16, 32, w, 6, outdir,
             script=[[31, 3, 7, 12, 20, 25]], seed=2)
    # wrapped ring (head != 0) with N-1 drawn -> next idx wraps to 0
    w = writes_random(rng, 45, 16)
    run_case("s16_wrapped", 16, 32, w, 8, outdir,
             script=[[31, 0, 5, 9, 17, 22, 28, 30]], seed=3)
    # redraw: first draw contains head-1 -> the reference draws again
    w = writes_random(rng, 20, 16)
    run_case("s16_redraw", 16, 64, w, 4, outdir,
             script=[[19, 1, 2, 3], [4, 0, 10, 2]], seed=4)
    # stale terminal slots: every other write terminal, never-written slots zero
    w = [(i % 4, (i % 3) - 1, None if i % 2 else rng.integers(0, 256, (4, 16, 16)).astype(np.uint8))
         for i in range(24)]
    run_case("s16_terminal", 16, 64, w, 10, outdir, seed=5)
    # B >= valid -> ValueError
    run_case("s16_too_small", 16, 64, writes_random(rng, 5, 16), 5, outdir, seed=6)
    # deepq64-sized slots (config 2 frame size)
    run_case("s64_basic", 64, 40, writes_random(rng, 38, 64), 32, outdir, seed=7)
    # one-hot of every action value, rewards spanning int16 sign
    w = [(i % 4, [-32768, -1, 0, 1, 32767][i % 5],
          rng.integers(0, 256, (4, 16, 16)).astype(np.uint8)) for i in range(30)]
    run_case("s16_extremes", 16, 40, w, 12, outdir, seed=8)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "tests/golden")
