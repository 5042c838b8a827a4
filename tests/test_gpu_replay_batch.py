"""GPU: large-batch replay sampling + Caffe-layout gather.

Bit-exact against the reference fixtures (tests/golden/replay_*.npz, made by
the reference's own replay.py) and the oracle's gather; the device draw is
checked for the selection semantics of replay.py:147-166 (sorted, distinct,
in [0, valid), never head-1, uniform); the 1M-slot, n = 32768 case is
checked through a size-independent property (tiled ring: every gathered row
equals its pool entry).
"""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ddq():
    import ddq as m
    return m


@pytest.fixture(scope="module")
def ref():
    from oracle import ref_numpy
    return ref_numpy


def host(bufs):
    return {k: v.cpu().numpy() for k, v in bufs.items()}


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(
    os.path.dirname(__file__), "golden", "replay_*.npz"))))
def test_batch_gather_bitexact_vs_reference(ddq, path):
    import torch
    f = np.load(path)
    S, N, B = int(f["S"]), int(f["N"]), int(f["B"])
    if str(f["error"]):
        pytest.skip("fixture encodes the B >= valid error (covered by the step gather test)")
    net = ddq.DeepQNet(batch=4, frame=S)
    net.replay_create(N)
    net.replay_import(f["st"], f["action"], f["reward"], f["non_terminal"].astype(np.uint8),
                      int(f["head"]), int(f["valid"]))
    bufs = net.batch_buffers(B)
    bufs["idx"].copy_(torch.from_numpy(f["idx"].astype(np.int32)))
    net.replay_gather_batch(bufs)
    out = host(bufs)
    np.testing.assert_array_equal(out["state"], f["out_state"])
    np.testing.assert_array_equal(out["next_state"], f["out_next_state"])
    np.testing.assert_array_equal(out["action"], f["out_action"])
    np.testing.assert_array_equal(out["reward"], f["out_reward"])
    np.testing.assert_array_equal(out["non_terminal"], f["out_non_terminal"])
    net.close()


@pytest.mark.parametrize("head", [0, 1234])
def test_batch_sampler_semantics_and_gather(ddq, ref, head):
    S, N, n = 16, 5000, 2000
    rng = np.random.default_rng(head)
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    ac = rng.integers(0, 4, N).astype(np.uint8)
    rw = rng.integers(-1, 2, N).astype(np.int16)
    nt = rng.random(N) > 0.1
    net = ddq.DeepQNet(batch=4, frame=S)
    net.replay_create(N)
    net.replay_import(st, ac, rw, nt.astype(np.uint8), head, N)
    r = ref.ReplayRef((4, S, S), N)
    r.state, r.action, r.reward, r.non_terminal = st, ac, rw, nt
    r.head, r.valid = head, N
    bufs = net.batch_buffers(n)
    seen_last = False
    prev = None
    for it in range(5):
        net.replay_sample_batch(bufs, seed=77)
        out = host(bufs)
        idx = out["idx"].astype(np.int64)
        assert idx.size == n and np.all(np.diff(idx) > 0)
        assert idx.min() >= 0 and idx.max() < N
        assert (head - 1) not in idx
        seen_last |= bool(idx[-1] == N - 1)
        s_ref, a_ref, r_ref, ns_ref, nt_ref = r.gather(idx)
        np.testing.assert_array_equal(out["state"], s_ref)
        np.testing.assert_array_equal(out["next_state"], ns_ref)
        np.testing.assert_array_equal(out["action"], a_ref)
        np.testing.assert_array_equal(out["reward"], r_ref)
        np.testing.assert_array_equal(out["non_terminal"], nt_ref)
        assert prev is None or not np.array_equal(prev, idx)   # the stream advances
        prev = idx
    if head == 0:
        assert seen_last          # 2000/5000 per draw: N-1 (wraps to slot 0) shows up
    net.close()


@pytest.mark.parametrize("S", [24, 40])
def test_batch_gather_partial_row_slices(ddq, ref, S):
    """The gather cuts a slot's S*S 4-byte words into 512-word slices a
    workgroup: at S = 24 / 40 (576 / 1600 words) the last slice is partial.
    Bit-exact against the oracle's gather of the same draw."""
    N, n = 700, 150
    rng = np.random.default_rng(S)
    st = rng.integers(0, 256, (N, 4, S, S)).astype(np.uint8)
    ac = rng.integers(0, 4, N).astype(np.uint8)
    rw = rng.integers(-1, 2, N).astype(np.int16)
    nt = rng.random(N) > 0.1
    net = ddq.DeepQNet(batch=4, frame=S)
    net.replay_create(N)
    net.replay_import(st, ac, rw, nt.astype(np.uint8), 0, N)
    r = ref.ReplayRef((4, S, S), N)
    r.state, r.action, r.reward, r.non_terminal = st, ac, rw, nt
    r.head, r.valid = 0, N
    bufs = net.batch_buffers(n)
    for _ in range(3):
        net.replay_sample_batch(bufs, seed=9)
        out = host(bufs)
        s_ref, a_ref, r_ref, ns_ref, nt_ref = r.gather(out["idx"].astype(np.int64))
        np.testing.assert_array_equal(out["state"], s_ref)
        np.testing.assert_array_equal(out["next_state"], ns_ref)
        np.testing.assert_array_equal(out["action"], a_ref)
        np.testing.assert_array_equal(out["reward"], r_ref)
        np.testing.assert_array_equal(out["non_terminal"], nt_ref)
    net.close()


def test_batch_sampler_uniform(ddq):
    """Chi-square of per-slot hit counts over many draws (valid=512, n=128)."""
    S, N, n, draws = 16, 512, 128, 400
    net = ddq.DeepQNet(batch=4, frame=S)
    net.replay_create(N)
    z = np.zeros((1, 4, S, S), np.uint8)
    net.replay_fill_tiled(z, np.zeros(1, np.uint8), np.zeros(1, np.int16), np.ones(1, np.uint8),
                          100, N)
    bufs = net.batch_buffers(n)
    counts = np.zeros(N)
    for _ in range(draws):
        net.replay_sample_batch(bufs, seed=5, check=False)
        counts[bufs["idx"].cpu().numpy()] += 1
    net._check(net.lib.ddq_replay_status(net.ctx))
    assert counts[99] == 0
    c = np.delete(counts, 99)
    e = draws * n / (N - 1)
    chi2 = ((c - e) ** 2 / e).sum()
    # dof = 510, sd = sqrt(2*510) ~ 32: 6 sd bound
    assert chi2 < 510 + 6 * 32, chi2
    net.close()


def test_batch_sampler_rejects_bad_sizes(ddq):
    net = ddq.DeepQNet(batch=4, frame=16)
    net.replay_create(100)
    z = np.zeros((1, 4, 16, 16), np.uint8)
    net.replay_fill_tiled(z, np.zeros(1, np.uint8), np.zeros(1, np.int16), np.ones(1, np.uint8),
                          0, 100)
    with pytest.raises(ddq._lib.DDQError, match="Can't draw sample of size 100"):
        net.replay_sample_batch(net.batch_buffers(100), seed=1)
    with pytest.raises(ddq._lib.DDQError, match="n <= valid/2"):
        net.replay_sample_batch(net.batch_buffers(60), seed=1)
    net.close()


def test_c5_million_slot_gather_property(ddq):
    """1M-slot 64x64 ring (16.4 GB in HBM) tiled from a 97-transition pool;
    n = 32768 draw: every row equals its pool entry (size-independent)."""
    import torch
    S, N, n, pool = 64, 1 << 20, 32768, 97
    rng = np.random.default_rng(11)
    st = rng.integers(0, 256, (pool, 4, S, S)).astype(np.uint8)
    ac = rng.integers(0, 4, pool).astype(np.uint8)
    rw = rng.integers(-1, 2, pool).astype(np.int16)
    nt = (rng.random(pool) > 0.2).astype(np.uint8)
    net = ddq.DeepQNet(batch=4, frame=S)
    net.replay_create(N)
    head = 4321
    net.replay_fill_tiled(st, ac, rw, nt, head, N)
    bufs = net.batch_buffers(n)
    net.replay_sample_batch(bufs, seed=2024)
    dev = bufs["idx"].device
    idx = bufs["idx"].long()
    assert bool((idx[1:] > idx[:-1]).all()) and int(idx[0]) >= 0 and int(idx[-1]) < N
    assert not bool((idx == head - 1).any())
    nxt = torch.where(idx + 1 == N, torch.zeros_like(idx), idx + 1)
    pst = torch.from_numpy(st).to(dev)
    assert torch.equal(bufs["state"], pst[idx % pool].float())
    assert torch.equal(bufs["next_state"], pst[nxt % pool].float())
    pac = torch.from_numpy(ac.astype(np.int64)).to(dev)[nxt % pool]
    assert torch.equal(bufs["action"].view(n, 4).argmax(1), pac)
    assert torch.equal(bufs["action"].sum(dim=(1, 2, 3)), torch.ones(n, device=dev))
    assert torch.equal(bufs["reward"].view(n),
                       torch.from_numpy(rw.astype(np.float32)).to(dev)[nxt % pool])
    assert torch.equal(bufs["non_terminal"].view(n),
                       torch.from_numpy(nt.astype(np.float32)).to(dev)[nxt % pool])
    net.close()
