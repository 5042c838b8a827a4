"""ORACLE fixture generator -- test infrastructure only.

Imports the REFERENCE expgain.py (read in place from /root/reference; it is
Python-2/3 compatible) and records golden vectors for the epsilon schedule
(expgain.py:55-60) and the nearest-neighbour preprocessor (expgain.py:12-27)
applied to gray-scaled Snake boards:

    python oracle/gen_expgain_golden.py tests/golden
"""
import os
import sys

import numpy as np

sys.dont_write_bytecode = True   # never write into the read-only reference tree
sys.path.insert(0, "/root/reference")
import expgain as ref_expgain  # noqa: E402  (the reference module itself)


def main(outdir):
    iters = np.array([0, 1, 100, 12345, 25000, 49999, 50000, 50001, 10 ** 6], np.int64)
    eg = ref_expgain.ExpGain(None, ["w", "a", "s", "d"], None, None, None, np.zeros((10, 10)))
    eps = np.array([eg.get_epsilon(int(i)) for i in iters], np.float64)
    rng = np.random.default_rng(0)
    boards = rng.integers(-2, 6, size=(3, 4, 10, 10)).astype(np.int64)   # codes -2..5
    gray = np.zeros(boards.shape, np.uint8)
    gray[boards != -1] = 200
    gray[boards == -2] = 255
    out = {"iters": iters, "epsilon": eps, "boards": boards, "gray": gray}
    for S in (16, 24, 64):
        f = ref_expgain.resampler((S, S))
        out["zoom%d" % S] = np.stack([f(g) for g in gray])
    np.savez_compressed(os.path.join(outdir, "expgain.npz"), **out)
    print("wrote", os.path.join(outdir, "expgain.npz"))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "tests/golden")
