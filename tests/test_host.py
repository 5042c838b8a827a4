"""CPU tests of the host-side drop-ins (no GPU needed): message byte format,
prototxt parsing, index draw vs the reference's recorded draws, Snake rules."""
import os
import pickle
import random
import struct

import numpy as np
import pytest

from oracle import ref_numpy as ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_model_message_bytes_match_restatement():
    from ddq.barista import messaging
    p = ref.init_params(16, seed=3)
    assert messaging.create_message(p, 17) == ref.create_message_ref(p, 17)


def test_gradient_message_roundtrip_and_layout():
    from ddq.barista import messaging
    p = ref.init_params(16, seed=4)
    p.update(ref.init_params(16, seed=5, prefix="P"))
    msg = messaging.create_net_message(p, "diff")
    (hlen,) = struct.unpack("i", msg[:4])
    header = pickle.loads(msg[4:4 + hlen])
    assert list(header) == ["Qconv1", "Qconv2", "Qconv3", "Qfc4", "Q_out"]   # Q* only
    assert header["Qconv1"] == [(32, 4, 7, 7), (1, 1, 1, 32)]
    assert len(msg) == 4 + hlen + 4 * ref.num_params(16)
    g = messaging.load_gradient_message(msg)
    r = ref.load_gradient_message_ref(msg)
    for k in g:
        for a, b, c in zip(g[k], r[k], p[k]):
            np.testing.assert_array_equal(a, b)
            np.testing.assert_array_equal(a, c)


def test_message_compression_roundtrip():
    from ddq.barista import messaging
    p = ref.init_params(16, seed=6)
    g = messaging.load_gradient_message(messaging.create_net_message(p, "diff", compress=True),
                                        compressed=True)
    np.testing.assert_array_equal(g["Qfc4"][0], p["Qfc4"][0])


def test_header_is_python2_readable_protocol():
    from ddq.barista import messaging
    msg = messaging.create_message(ref.init_params(16), 0)
    hlen = struct.unpack("ii", msg[:8])[1]
    assert msg[8:10] == b"\x80\x02"          # pickle protocol 2 (cPickle -1 in Py2)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /dev/null",))


@pytest.mark.parametrize("kind", ["model", "gradient"])
def test_malicious_header_is_refused(kind, monkeypatch):
    """Headers come off the network: a pickle naming any global but
    OrderedDict is refused before anything runs (messaging.py:89)."""
    from ddq.barista import messaging
    header = pickle.dumps(collections_od([("Qconv1", _Evil())]), 2)   # names os.system
    called = []
    monkeypatch.setattr(os, "system", lambda *a: called.append(a))
    data = np.zeros(4, np.float32).tobytes()
    if kind == "model":
        msg = struct.pack("ii", 0, len(header)) + header + data
        with pytest.raises(pickle.UnpicklingError):
            messaging.load_model_params(msg)
    else:
        msg = struct.pack("i", len(header)) + header + data
        with pytest.raises(pickle.UnpicklingError):
            messaging.load_gradient_message(msg)
    assert not called
    # a malformed (but harmless) header is rejected too
    bad = pickle.dumps({"Qconv1": "not shapes"}, 2)
    with pytest.raises(ValueError):
        messaging.load_gradient_message(struct.pack("i", len(bad)) + bad + data)


def test_python2_style_header_still_loads():
    """A header as Python 2 cPickle.dumps(OrderedDict, -1) writes it (str names
    as SHORT_BINSTRING, tuples of ints) decodes with the restricted loader."""
    from ddq.barista import messaging
    # protocol-2 pickle of OrderedDict([('Qconv1', [(2, 2), (1, 1, 1, 2)])]) with
    # Python 2 byte strings ('U' opcodes), as cPickle writes it
    raw = (b"\x80\x02ccollections\nOrderedDict\nq\x00)Rq\x01U\x06Qconv1q\x02]q\x03"
           b"(K\x02K\x02\x86q\x04(K\x01K\x01K\x01K\x02tq\x05es.")
    data = np.arange(6, dtype=np.float32).tobytes()
    g = messaging.load_gradient_message(struct.pack("i", len(raw)) + raw + data)
    assert list(g) == ["Qconv1"]
    np.testing.assert_array_equal(g["Qconv1"][0], [[0, 1], [2, 3]])
    np.testing.assert_array_equal(g["Qconv1"][1].ravel(), [4, 5])


def collections_od(items):
    import collections
    return collections.OrderedDict(items)


def test_parse_architecture():
    from ddq.barista.baristanet import parse_architecture
    assert parse_architecture(os.path.join(GOLD, "deepq16.prototxt")) == (32, 16, 0.85)
    assert parse_architecture({"batch": 8, "frame": 64}) == (8, 64, 0.85)


@pytest.mark.parametrize("name,seed", [("s16_basic", 1), ("s16_terminal", 5), ("s64_basic", 7),
                                       ("s16_extremes", 8)])
def test_index_draw_matches_reference_draws(name, seed):
    """With Python's random seeded as the fixture generator did, the drop-in's
    host index draw (random.sample + head-1 redraw + sort) reproduces the
    reference's recorded list, redraws included."""
    f = np.load(os.path.join(GOLD, "replay_%s.npz" % name))
    head, valid, B = int(f["head"]), int(f["valid"]), int(f["B"])

    class Ring:            # only what draw_indices reads
        def replay_info(self):
            return head, valid, int(f["N"])
    from ddq.replay import ReplayDataset
    ds = ReplayDataset.__new__(ReplayDataset)
    ds._net = Ring()
    random.seed(seed)
    idx = ds.draw_indices(B)
    np.testing.assert_array_equal(idx, f["idx"])


def test_snake_rules():
    from ddq.snake import SnakeGame, EMPTY, APPLE
    g = SnakeGame(random.Random(0))
    s = g.encode_state()
    assert s[6, 5] == 0 and s[5, 5] == 1 and (s == APPLE).sum() == 1
    # moving west (opposite of the east heading) keeps heading east
    ns, r, over = g.cpu_play(s, "a")
    assert not over and ns[7, 5] == 0 and ns[6, 5] == 1 and (ns >= 0).sum() == 2
    # run into the east wall
    st = ns
    for _ in range(5):
        st, r, over = g.cpu_play(st, "d")
        if over:
            break
    assert over and r == -1


def test_synthetic_transitions_shapes():
    from ddq.expgain import synthetic_transitions
    st, ac, rw, nt = synthetic_transitions(64, 16, seed=1)
    assert st.shape == (64, 4, 16, 16) and st.dtype == np.uint8
    assert set(np.unique(st)) <= {0, 200, 255}
    assert set(np.unique(rw)) <= {-1, 0, 1}
    assert (~nt).sum() == (rw == -1).sum()
