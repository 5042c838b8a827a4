"""Replay file format: ddq.h5lite against files the
reference's own replay.py wrote and read (fixtures: oracle/gen_hdf5_golden.py),
and -- where /opt/conda/bin/python3.9 has h5py (this container) -- against
h5py directly."""
import os
import subprocess

import numpy as np
import pytest

from ddq import h5lite

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
H5PY = "/opt/conda/bin/python3.9"


def have_h5py():
    if not os.path.exists(H5PY):
        return False
    return subprocess.run([H5PY, "-c", "import h5py"], capture_output=True).returncode == 0


def ring_equal(got, want, pre=""):
    for k in ("state", "action", "reward", "non_terminal"):
        np.testing.assert_array_equal(got[k], want[pre + k], err_msg=k)
        assert got[k].dtype == want[pre + k].dtype, k
    assert int(got["head"]) == int(want[pre + "head"])
    assert int(got["valid"]) == int(want[pre + "valid"])


def test_reads_file_written_by_reference():
    want = np.load(os.path.join(GOLD, "h5_ref_s16.npz"))
    got = h5lite.read_replay(os.path.join(GOLD, "h5_ref_s16.hdf5"))
    ring_equal(got, want)
    # the ring wrapped (15 writes, 12 slots) and holds terminal slots
    assert got["head"] == 3 and got["valid"] == 12 and not got["non_terminal"].all()


def test_writer_output_is_what_the_reference_read():
    """The reference reopened write_replay's output and read back exactly the
    inputs (fixture); the writer is deterministic, so the bytes pin it."""
    f = np.load(os.path.join(GOLD, "h5_resume.npz"))
    for k in ("state", "action", "reward", "non_terminal", "head", "valid"):
        np.testing.assert_array_equal(f["read_" + k], f["in_" + k])
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "w.hdf5")
        h5lite.write_replay(p, f["in_state"], f["in_action"], f["in_reward"],
                            f["in_non_terminal"], int(f["in_head"]), int(f["in_valid"]))
        assert open(p, "rb").read() == open(os.path.join(GOLD, "h5_resume_in.hdf5"),
                                            "rb").read()


def test_reads_file_the_reference_resumed_and_persisted():
    f = np.load(os.path.join(GOLD, "h5_resume.npz"))
    got = h5lite.read_replay(os.path.join(GOLD, "h5_resume_out.hdf5"))
    ring_equal(got, f, "fin_")


def test_round_trip_and_fill_callback(tmp_path):
    rng = np.random.default_rng(3)
    N, S = 257, 24
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    ac = rng.integers(0, 4, N).astype(np.uint8)
    rw = rng.integers(-32768, 32768, N).astype(np.int16)
    nt = rng.random(N) < 0.5
    p = str(tmp_path / "r.hdf5")
    h5lite.write_replay(p, st, ac, rw, nt, 100, 257)
    got = h5lite.read_replay(p, mmap_state=True)
    assert isinstance(got["state"], np.memmap)
    ring_equal(got, dict(state=st, action=ac, reward=rw, non_terminal=nt, head=100, valid=257))

    def fill(mm):
        mm[...] = st
        return ac, rw, nt
    p2 = str(tmp_path / "r2.hdf5")
    h5lite.write_replay(p2, fill, head=100, valid=257, shape=st.shape)
    assert open(p, "rb").read() == open(p2, "rb").read()
    # the state block is 4 KiB aligned (memory-mapped fills)
    assert h5lite.H5File(p).datasets["state"].addr % 4096 == 0


def test_bad_inputs(tmp_path):
    p = str(tmp_path / "x.hdf5")
    with pytest.raises(h5lite.H5Error):
        h5lite.write_replay(p, np.zeros((4, 4, 2, 2), np.uint8), np.zeros(3, np.uint8),
                            np.zeros(4, np.int16), np.zeros(4, bool), 0, 0)
    assert not os.path.exists(p)
    open(p, "wb").write(b"not an hdf5 file" * 10)
    with pytest.raises(h5lite.H5Error):
        h5lite.read_replay(p)


@pytest.mark.skipif(not have_h5py(), reason="no h5py interpreter in this image")
def test_h5py_reads_writer_output_and_appends(tmp_path):
    rng = np.random.default_rng(5)
    N, S = 33, 16
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    ac = rng.integers(0, 4, N).astype(np.uint8)
    rw = rng.integers(-5, 6, N).astype(np.int16)
    nt = rng.random(N) < 0.6
    p = str(tmp_path / "w.hdf5")
    h5lite.write_replay(p, st, ac, rw, nt, 17, 30)
    np.savez(str(tmp_path / "e.npz"), st=st, ac=ac, rw=rw, nt=nt)
    code = r"""
import sys, h5py, numpy as np
e = np.load(sys.argv[2]); f = h5py.File(sys.argv[1], "r")
assert sorted(f.keys()) == ["action", "non_terminal", "reward", "state"]
assert f["non_terminal"].dtype == bool and f["reward"].dtype == np.int16
assert (f["state"][...] == e["st"]).all() and (f["action"][...] == e["ac"]).all()
assert (f["reward"][...] == e["rw"]).all() and (f["non_terminal"][...] == e["nt"]).all()
assert int(f["state"].attrs["head"]) == 17 and int(f["state"].attrs["valid"]) == 30
f.close()
f = h5py.File(sys.argv[1], "a")        # what the reference does on resume + persist
f["action"][:] = 3; f["state"][0] = 9; f["state"].attrs["head"] = 5
f.create_dataset("extra", (2,), dtype="f4"); f.close()
"""
    r = subprocess.run([H5PY, "-c", code, p, str(tmp_path / "e.npz")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    got = h5lite.read_replay(p)
    assert got["head"] == 5 and (got["action"] == 3).all() and (got["state"][0] == 9).all()
    np.testing.assert_array_equal(got["state"][1:], st[1:])


@pytest.mark.skipif(not have_h5py(), reason="no h5py interpreter in this image")
@pytest.mark.parametrize("libver", ["earliest", "latest"])
def test_reads_h5py_files(tmp_path, libver):
    p = str(tmp_path / "h.hdf5")
    code = r"""
import sys, h5py, numpy as np
rng = np.random.default_rng(9)
f = h5py.File(sys.argv[1], "w", libver=sys.argv[2])
s = f.create_dataset("state", (7, 4, 8, 8), dtype="uint8")
s[2:5] = rng.integers(0, 256, (3, 4, 8, 8))
f.create_dataset("action", data=np.arange(7, dtype=np.uint8))
f.create_dataset("reward", data=np.array([-1, 0, 1, 2, -32768, 32767, 5], np.int16))
f.create_dataset("non_terminal", data=np.array([1, 0, 1, 1, 0, 1, 1], bool))
s.attrs["head"] = 0; s.attrs["valid"] = 0
s.attrs["head"] = np.int64(5); s.attrs["valid"] = 6
np.save(sys.argv[1] + ".npy", s[...]); f.close()
"""
    r = subprocess.run([H5PY, "-c", code, p, libver], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = h5lite.read_replay(p)
    np.testing.assert_array_equal(got["state"], np.load(p + ".npy"))
    np.testing.assert_array_equal(got["reward"], [-1, 0, 1, 2, -32768, 32767, 5])
    np.testing.assert_array_equal(got["non_terminal"], [1, 0, 1, 1, 0, 1, 1])
    assert got["head"] == 5 and got["valid"] == 6 and got["action"].tolist() == list(range(7))


@pytest.mark.skipif(not have_h5py(), reason="no h5py interpreter in this image")
def test_rejects_chunked_storage(tmp_path):
    p = str(tmp_path / "c.hdf5")
    code = r"""
import sys, h5py, numpy as np
f = h5py.File(sys.argv[1], "w")
f.create_dataset("state", (4, 4, 2, 2), dtype="uint8", chunks=(1, 4, 2, 2))
for n, t in (("action", "uint8"), ("reward", "int16"), ("non_terminal", bool)):
    f.create_dataset(n, (4,), dtype=t)
f.close()
"""
    r = subprocess.run([H5PY, "-c", code, p], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    with pytest.raises(h5lite.H5Error, match="chunked"):
        h5lite.read_replay(p)


@pytest.mark.skipif(not have_h5py(), reason="no h5py interpreter in this image")
def test_missing_datasets_mean_create(tmp_path):
    """A file without the replay datasets -> None: the reference then creates
    them (replay.py:29, :47-62)."""
    p = str(tmp_path / "e.hdf5")
    r = subprocess.run([H5PY, "-c", "import sys, h5py; f = h5py.File(sys.argv[1], 'w'); "
                        "f.create_dataset('other', (3,), dtype='f4'); f.close()", p],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert h5lite.read_replay(p) is None
    assert list(h5lite.H5File(p).datasets) == ["other"]
