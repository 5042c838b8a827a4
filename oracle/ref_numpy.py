"""ORACLE -- test infrastructure only.  NOT product code.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the *checker*.  The shipped path
(``distributed-deep-q_amd/ddq``) never imports it; it fails loudly when the HIP
library is missing.

A float64 numpy restatement of the reference's data-parallel DQN step:

* replay ring write / minibatch gather ........ replay.py:70-92, :144-183
* deepq network forward (Q and frozen P) ...... models/deepq/train_val.prototxt:38-383
* Q(s,a) mask-select, Bellman target, loss .... train_val.prototxt:385-483
* Q-net backward (Caffe 2014 layer semantics) . absent ``caffe`` submodule, see below
* param-server apply rules + target sync ...... param-server/server.py:49-137
* Caffe SGDSolver momentum (solver.prototxt) .. solver.prototxt:4-11 (not used by the
  reference's distributed path -- SURVEY.md finding 3)

Pinning status
--------------
* Replay gather/ring semantics: PINNED against the reference's own
  ``replay.py`` executed in this container (``oracle/gen_replay_golden.py``
  -> ``tests/golden/replay_*.npz``).
* Parameter layout (names, Caffe 4-D shapes, pycaffe order): pinned by the
  reference's published parameter counts, results/cost-vs-image-size-trials.txt
  column 6 (228,132 ... 8,485,668 for 16..128 px).
* Network arithmetic (conv / pool / IP / eltwise / Euclidean loss forward and
  backward): the algorithm lives in the un-vendored third-party submodule
  ``caffe`` -> https://github.com/kjchavez/caffe.git (.gitmodules:1-3), pinned
  commit unknown (gitlink absent), a mid-2014 Caffe (V1 ``layers{}`` syntax,
  global ``set_phase_test``).  It cannot be built here.  The restatement
  follows Caffe's published layer algorithms (im2col convolution, MAX pooling
  with first-max argmax, in-place ReLU, TEST-phase dropout = identity,
  EuclideanLoss = sum(d^2)/(2N)).  The reference's own tests pin nothing at this
  boundary -> **parity unpinned** for the network arithmetic; mitigated by an
  independent torch-CPU float64 implementation in tests/test_oracle.py.
* Update rules / messaging byte layout: the reference modules are Python-2 only
  (print statements, cPickle, urllib2) and cannot be imported; restated from
  the source text -> parity unpinned (checked by reading, cited per function).
"""
from __future__ import annotations

import collections
import pickle
import struct

import numpy as np

GAMMA = 0.85          # train_val.prototxt:473 (coeff of P_sa in target_Q_sa)
NUM_ACTIONS = 4       # barista/constants.py:8
NFRAME = 4            # expgain.py:9, train_val.prototxt:9
EPS = 1e-8            # server.py:105,124 (inside the sqrt)

# (name, Cout, kernel, pad) of the three convolutions, train_val.prototxt:39-141
CONVS = (("conv1", 32, 7, 3), ("conv2", 64, 5, 2), ("conv3", 64, 3, 1))
FC4 = 512             # train_val.prototxt:169
# gaussian filler std per layer, train_val.prototxt:52-55,92-95,132-135,170-173,206-209
FILLER_STD = {"conv1": 0.01, "conv2": 0.01, "conv3": 0.01, "fc4": 0.005, "_out": 0.01}


# --------------------------------------------------------------------------
# parameter layout (pycaffe net.params order)
# --------------------------------------------------------------------------
def layer_names(prefix):
    """Layer names in prototxt order: Qconv1..Q_out (train_val.prototxt:39-215)."""
    return [prefix + "conv1", prefix + "conv2", prefix + "conv3",
            prefix + "fc4", prefix + "_out"]


def param_shapes(S, prefix="Q"):
    """Caffe-2014 4-D blob shapes of each layer's [weight, bias].

    conv W (Cout,Cin,k,k), conv/IP bias (1,1,1,Cout), IP W (1,1,out,in)
    (element counts pinned by
    results/cost-vs-image-size-trials.txt column 6).
    """
    assert S % 8 == 0, "frame side must be a multiple of 8"
    s4 = S // 8
    cin = NFRAME
    out = collections.OrderedDict()
    names = layer_names(prefix)
    for (nm, cout, k, _), lname in zip(CONVS, names[:3]):
        out[lname] = [(cout, cin, k, k), (1, 1, 1, cout)]
        cin = cout
    out[names[3]] = [(1, 1, FC4, 64 * s4 * s4), (1, 1, 1, FC4)]
    out[names[4]] = [(1, 1, NUM_ACTIONS, FC4), (1, 1, 1, NUM_ACTIONS)]
    return out


def num_params(S):
    return sum(int(np.prod(s)) for v in param_shapes(S).values() for s in v)


def init_params(S, seed=42, prefix="Q"):
    """Gaussian fillers (std per train_val.prototxt), bias 0 (constant filler)."""
    rng = np.random.default_rng(seed)
    p = collections.OrderedDict()
    for lname, (ws, bs) in param_shapes(S, prefix).items():
        std = FILLER_STD[lname[1:]]
        p[lname] = [rng.normal(0.0, std, size=ws).astype(np.float32),
                    np.zeros(bs, np.float32)]
    return p


def flatten(params):
    return np.concatenate([b.ravel() for v in params.values() for b in v])


def unflatten(flat, S, prefix="Q"):
    out = collections.OrderedDict()
    o = 0
    for lname, shapes in param_shapes(S, prefix).items():
        out[lname] = []
        for s in shapes:
            n = int(np.prod(s))
            out[lname].append(np.asarray(flat[o:o + n]).reshape(s))
            o += n
    return out


# --------------------------------------------------------------------------
# Caffe layer semantics (float64)
# --------------------------------------------------------------------------
def im2col(x, k, pad):
    """Caffe im2col: rows ordered (c, ky, kx), columns (y, x); x is (C,H,W)."""
    C, H, W = x.shape
    xp = np.zeros((C, H + 2 * pad, W + 2 * pad), x.dtype)
    xp[:, pad:pad + H, pad:pad + W] = x
    cols = np.empty((C, k, k, H, W), x.dtype)
    for ky in range(k):
        for kx in range(k):
            cols[:, ky, kx] = xp[:, ky:ky + H, kx:kx + W]
    return cols.reshape(C * k * k, H * W)


def col2im(cols, C, H, W, k, pad):
    """Caffe col2im (adjoint of im2col)."""
    c = cols.reshape(C, k, k, H, W)
    xp = np.zeros((C, H + 2 * pad, W + 2 * pad), cols.dtype)
    for ky in range(k):
        for kx in range(k):
            xp[:, ky:ky + H, kx:kx + W] += c[:, ky, kx]
    return xp[:, pad:pad + H, pad:pad + W]


def conv_forward(x, W, b, pad):
    """CONVOLUTION: top = W.reshape(Cout,K) @ im2col(x) + bias (per image)."""
    B, C, H, Wd = x.shape
    cout, _, k, _ = W.shape
    Wm = W.reshape(cout, -1)
    top = np.empty((B, cout, H, Wd), np.float64)
    for n in range(B):
        top[n] = (Wm @ im2col(x[n], k, pad)).reshape(cout, H, Wd)
    return top + b.reshape(1, cout, 1, 1)


def conv_backward(x, W, top_diff, pad, need_bottom=True):
    """Caffe ConvolutionLayer::Backward: weight diff zeroed then summed over
    images; bias diff = sum over (n, y, x); bottom diff via col2im."""
    B, C, H, Wd = x.shape
    cout, _, k, _ = W.shape
    Wm = W.reshape(cout, -1)
    dW = np.zeros_like(Wm, dtype=np.float64)
    dx = np.zeros(x.shape, np.float64) if need_bottom else None
    for n in range(B):
        td = top_diff[n].reshape(cout, -1)
        dW += td @ im2col(x[n], k, pad).T
        if need_bottom:
            dx[n] = col2im(Wm.T @ td, C, H, Wd, k, pad)
    db = top_diff.sum(axis=(0, 2, 3))
    return dW.reshape(W.shape), db, dx


def relu(x):
    return np.maximum(x, 0.0)


def maxpool_forward(x):
    """MAX pooling 2x2 stride 2 (Caffe): argmax = FIRST max in row-major window
    order (comparison ``>`` starting from -FLT_MAX).  Returns top and the
    flat in-window argmax (0..3)."""
    B, C, H, W = x.shape
    assert H % 2 == 0 and W % 2 == 0
    win = x.reshape(B, C, H // 2, 2, W // 2, 2).transpose(0, 1, 2, 4, 3, 5)
    win = win.reshape(B, C, H // 2, W // 2, 4)
    arg = np.argmax(win, axis=-1)           # numpy argmax = first max
    top = np.take_along_axis(win, arg[..., None], -1)[..., 0]
    return top, arg


def maxpool_backward(top_diff, arg, H, W):
    B, C, Hp, Wp = top_diff.shape
    win = np.zeros((B, C, Hp, Wp, 4), np.float64)
    np.put_along_axis(win, arg[..., None], top_diff[..., None], -1)
    win = win.reshape(B, C, Hp, Wp, 2, 2).transpose(0, 1, 2, 4, 3, 5)
    return win.reshape(B, C, H, W)


def net_forward(x, p, prefix="Q"):
    """Forward of one tower (train_val.prototxt:38-215 / :216-383).

    Dropout is identity: main.py:147 sets the TEST phase before the net is
    built (SURVEY.md finding 4).  Returns every intermediate needed by the
    backward pass."""
    names = layer_names(prefix)
    cache = {"x0": x}
    h = x
    for i, ((_, _, k, pad), lname) in enumerate(zip(CONVS, names[:3])):
        W, b = p[lname]
        pre = conv_forward(h, W, b.reshape(-1), pad)
        act = relu(pre)                     # RELU in place
        top, arg = maxpool_forward(act)
        cache["x%d" % i] = h
        cache["act%d" % (i + 1)] = act
        cache["arg%d" % (i + 1)] = arg
        h = top
    cache["pool3"] = h
    B = x.shape[0]
    flat = h.reshape(B, -1)                 # NCHW flatten: c*S4^2 + y*S4 + x
    W4, b4 = p[names[3]]
    pre4 = flat @ W4.reshape(FC4, -1).T + b4.reshape(-1)
    h4 = relu(pre4)
    W5, b5 = p[names[4]]
    out = h4 @ W5.reshape(NUM_ACTIONS, -1).T + b5.reshape(-1)
    cache.update(flat=flat, pre4=pre4, h4=h4, out=out)
    return cache


def route_codes(act, arg):
    """Routing byte per pooled element: first-max position 0..3, or 4 when the
    window max is <= 0 (ReLU in place => no gradient reaches the window)."""
    B, C, H, W = act.shape
    win = act.reshape(B, C, H // 2, 2, W // 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(
        B, C, H // 2, W // 2, 4)
    return np.where(win.max(-1) > 0, arg, 4).astype(np.uint8)


def full_pass(pQ, pP, state, action, reward, next_state, non_terminal, routes=None,
              return_cache=False, h4_mask=None):
    """BaristaNet.full_pass (baristanet.py:138-140) = net.forward(); net.backward().

    Inputs in the reference's MEMORY_DATA shapes: state/next_state (B,4,S,S),
    action (B,4,1,1) one-hot, reward/non_terminal (B,1,1,1).  Returns the
    blobs (Q_out, P_out, Q_sa, P_sa, target_Q_sa, loss) and the Q-parameter
    diffs as an OrderedDict in pycaffe order."""
    f64 = lambda a: np.asarray(a, np.float64)
    state, next_state = f64(state), f64(next_state)
    B = state.shape[0]
    act = f64(action).reshape(B, NUM_ACTIONS)
    r = f64(reward).reshape(B)
    nt = f64(non_terminal).reshape(B)
    pQ = {k: [f64(w) for w in v] for k, v in pQ.items()}
    pP = {k: [f64(w) for w in v] for k, v in pP.items()}

    cq = net_forward(state, pQ, "Q")
    cp = net_forward(next_state, pP, "P")
    Q, P = cq["out"], cp["out"]
    q_sa = (Q * act).sum(axis=1)                    # :386-422 PROD, SLICE, SUM
    p_sa = P.max(axis=1) * nt                       # :429-464 SLICE, MAX, PROD
    target = GAMMA * p_sa + 1.0 * r                 # :465-476 SUM coeff 0.85, 1
    diff = q_sa - target
    loss = float(diff @ diff) / B / 2.0             # EUCLIDEAN_LOSS :477-483

    # ---- backward (Q tower only; P has blobs_lr 0 and data bottoms) ----
    dQ = act * (diff / B)[:, None]                  # loss -> SUM -> SLICE -> PROD
    names = layer_names("Q")
    grads = collections.OrderedDict()
    W5 = pQ[names[4]][0].reshape(NUM_ACTIONS, -1)
    h4 = cq["h4"]
    gW5 = dQ.T @ h4
    gb5 = dQ.sum(0)
    # IP bottom diff, ReLU mask (h4_mask: an externally decided fc4 ReLU mask,
    # the parity harness's adoption of the GPU's side of a proven near-tie)
    dh4 = (dQ @ W5) * ((h4 > 0) if h4_mask is None else h4_mask)
    W4 = pQ[names[3]][0].reshape(FC4, -1)
    flat = cq["flat"]
    gW4 = dh4.T @ flat
    gb4 = dh4.sum(0)
    dflat = dh4 @ W4
    dpool = dflat.reshape(cq["pool3"].shape)
    conv_grads = []
    for i in (3, 2, 1):
        act_i = cq["act%d" % i]
        if routes is None:
            dact = maxpool_backward(dpool, cq["arg%d" % i], act_i.shape[2], act_i.shape[3])
            dpre = dact * (act_i > 0)                # ReLU backward (in-place top > 0)
        else:
            # externally supplied routing (codes of route_codes); 4 = no gradient
            code = np.asarray(routes[i])
            keep = code < 4
            dpre = maxpool_backward(dpool * keep, np.where(keep, code, 0),
                                    act_i.shape[2], act_i.shape[3])
        W = pQ[names[i - 1]][0]
        gW, gb, dx = conv_backward(cq["x%d" % (i - 1)], W, dpre, CONVS[i - 1][3],
                                   need_bottom=(i > 1))
        conv_grads.append((gW, gb))
        dpool = dx
    conv_grads.reverse()
    shapes = param_shapes(state.shape[2], "Q")
    for (gW, gb), lname in zip(conv_grads, names[:3]):
        grads[lname] = [gW.reshape(shapes[lname][0]), gb.reshape(shapes[lname][1])]
    grads[names[3]] = [gW4.reshape(shapes[names[3]][0]), gb4.reshape(shapes[names[3]][1])]
    grads[names[4]] = [gW5.reshape(shapes[names[4]][0]), gb5.reshape(shapes[names[4]][1])]
    blobs = dict(Q_out=Q, P_out=P, Q_sa=q_sa, P_sa=p_sa, target_Q_sa=target, loss=loss)
    if return_cache:
        return blobs, grads, cq
    return blobs, grads


def magnitudes(pQ, pP, state, action, reward, next_state, non_terminal, routes=None,
               h4_mask=None):
    """Per-element magnitude M of every blob and gradient of ``full_pass``:
    the same computation with every operand replaced by its absolute value
    (|W|, |x|, |b|, |dQ| ...) along the same ReLU / max-pool routing.  M is the
    sum of |terms| an output element accumulates -- its condition: fp32
    rounding of the terms (and relative errors of the inputs) perturb the
    element by a small multiple of eps32 * M however much the terms cancel.
    The parity tests bound each element by rtol * |ref| + c * M (tests/_parity.py),
    an elementwise tolerance with no tensor-wide floor.  Returns
    (blob_mags, grad_mags) keyed like full_pass's outputs."""
    f64 = lambda a: np.abs(np.asarray(a, np.float64))
    B = np.asarray(state).shape[0]
    act = f64(action).reshape(B, NUM_ACTIONS)
    r = f64(reward).reshape(B)
    nt = f64(non_terminal).reshape(B)
    pQa = {k: [f64(w) for w in v] for k, v in pQ.items()}
    pPa = {k: [f64(w) for w in v] for k, v in pP.items()}
    # signed forward for the routing / ReLU decisions
    cq = net_forward(np.asarray(state, np.float64),
                     {k: [np.asarray(w, np.float64) for w in v] for k, v in pQ.items()}, "Q")
    cp = net_forward(np.asarray(next_state, np.float64),
                     {k: [np.asarray(w, np.float64) for w in v] for k, v in pP.items()}, "P")

    def fwd_mag(x, pa, cache, prefix, rts, m4=None):
        names = layer_names(prefix)
        h = f64(x)
        ins = []
        for i, ((_, _, k, pad), lname) in enumerate(zip(CONVS, names[:3])):
            W, b = pa[lname]
            ins.append(h)
            m_all = conv_forward(h, W, b.reshape(-1), pad)
            a_s = cache["act%d" % (i + 1)]
            m = np.where(a_s > 0, m_all, 0.0)
            if rts is not None and prefix == "Q":
                code = np.asarray(rts[i + 1])
                keep = code < 4
                # a routed window's value is the conv sum at the routed pixel,
                # whatever the float64 sign there: at an adopted near-tie (the
                # GPU's max a tiny positive fp32 value, the oracle's <= 0) its
                # magnitude is that sum's |terms|, not 0
                m = m_all
                win = m.reshape(B, m.shape[1], m.shape[2] // 2, 2, m.shape[3] // 2, 2).transpose(
                    0, 1, 2, 4, 3, 5).reshape(B, m.shape[1], m.shape[2] // 2, m.shape[3] // 2, 4)
                h = np.take_along_axis(win, np.where(keep, code, 0)[..., None], -1)[..., 0] * keep
            else:
                arg = cache["arg%d" % (i + 1)]
                win = m.reshape(B, m.shape[1], m.shape[2] // 2, 2, m.shape[3] // 2, 2).transpose(
                    0, 1, 2, 4, 3, 5).reshape(B, m.shape[1], m.shape[2] // 2, m.shape[3] // 2, 4)
                h = np.take_along_axis(win, arg[..., None], -1)[..., 0]
        flat = h.reshape(B, -1)
        W4, b4 = pa[names[3]]
        mh4 = (flat @ W4.reshape(FC4, -1).T + b4.reshape(-1)) * (
            (cache["h4"] > 0) if m4 is None else m4)
        W5, b5 = pa[names[4]]
        mout = mh4 @ W5.reshape(NUM_ACTIONS, -1).T + b5.reshape(-1)
        return ins, flat, mh4, mout

    mask4 = (cq["h4"] > 0) if h4_mask is None else h4_mask
    insq, mflat, mh4, mQ = fwd_mag(state, pQa, cq, "Q", routes, mask4)
    _, _, _, mP = fwd_mag(next_state, pPa, cp, "P", None)
    Q, P = cq["out"], cp["out"]
    m_qsa = (mQ * act).sum(axis=1)
    m_psa = mP[np.arange(B), P.argmax(axis=1)] * nt
    m_target = GAMMA * m_psa + r
    m_diff = m_qsa + m_target
    diff = np.abs((Q * np.asarray(action, np.float64).reshape(B, -1)).sum(1)
                  - (GAMMA * P.max(1) * np.asarray(non_terminal, np.float64).reshape(B)
                     + np.asarray(reward, np.float64).reshape(B)))
    m_loss = float((diff * m_diff).sum() / B)
    blobs = dict(Q_out=mQ, P_out=mP, Q_sa=m_qsa, P_sa=m_psa, target_Q_sa=m_target, loss=m_loss)
    # backward on magnitudes
    names = layer_names("Q")
    mdQ = act * (m_diff / B)[:, None]
    W5 = pQa[names[4]][0].reshape(NUM_ACTIONS, -1)
    g = collections.OrderedDict()
    gW5 = mdQ.T @ mh4                    # products of magnitudes bound both error terms
    gb5 = mdQ.sum(0)
    mdh4 = (mdQ @ W5) * mask4
    W4 = pQa[names[3]][0].reshape(FC4, -1)
    gW4 = mdh4.T @ mflat
    gb4 = mdh4.sum(0)
    dpool = (mdh4 @ W4).reshape(cq["pool3"].shape)
    conv_g = []
    for i in (3, 2, 1):
        act_i = cq["act%d" % i]
        if routes is None:
            dpre = maxpool_backward(dpool, cq["arg%d" % i], act_i.shape[2], act_i.shape[3])
            dpre = dpre * (act_i > 0)
        else:
            code = np.asarray(routes[i])
            keep = code < 4
            dpre = maxpool_backward(dpool * keep, np.where(keep, code, 0), act_i.shape[2],
                                    act_i.shape[3])
        W = pQa[names[i - 1]][0]
        gW, gb, dx = conv_backward(insq[i - 1], W, dpre, CONVS[i - 1][3], need_bottom=(i > 1))
        conv_g.append((gW, gb))
        dpool = dx
    conv_g.reverse()
    shapes = param_shapes(np.asarray(state).shape[2], "Q")
    for (gW, gb), lname in zip(conv_g, names[:3]):
        g[lname] = [gW.reshape(shapes[lname][0]), gb.reshape(shapes[lname][1])]
    g[names[3]] = [gW4.reshape(shapes[names[3]][0]), gb4.reshape(shapes[names[3]][1])]
    g[names[4]] = [gW5.reshape(shapes[names[4]][0]), gb5.reshape(shapes[names[4]][1])]
    return blobs, g


def select_action(state_f32, pQ):
    """BaristaNet.select_action (baristanet.py:142-146): argmax of Q_out (first max)."""
    return np.argmax(net_forward(np.asarray(state_f32, np.float64),
                                 {k: [np.asarray(w, np.float64) for w in v]
                                  for k, v in pQ.items()}, "Q")["out"], axis=1)


# --------------------------------------------------------------------------
# replay (replay.py)
# --------------------------------------------------------------------------
class ReplayRef:
    """Ring buffer with the exact field dtypes of replay.py:48-61."""

    def __init__(self, state_shape, dset_size):
        self.N = dset_size
        self.state = np.zeros((dset_size,) + tuple(state_shape), np.uint8)  # h5py fill 0
        self.action = np.zeros(dset_size, np.uint8)
        self.reward = np.zeros(dset_size, np.int16)
        self.non_terminal = np.zeros(dset_size, bool)
        self.head = 0
        self.valid = 0

    def add_experience(self, action, reward, state):
        """replay.py:70-92: terminal (state None) leaves state[head] stale."""
        self.action[self.head] = action
        self.reward[self.head] = reward
        if state is not None:
            self.state[self.head] = state
            self.non_terminal[self.head] = True
        else:
            self.non_terminal[self.head] = False
        self.head = (self.head + 1) % self.N
        self.valid = min(self.N, self.valid + 1)

    def gather(self, idx):
        """sample_direct (replay.py:159-183) given the drawn index list."""
        idx = sorted(int(i) for i in idx)
        nxt = [i + 1 for i in idx]
        if nxt[-1] == self.N:                          # only the last can wrap
            nxt[-1] = 0
        B = len(idx)
        state = self.state[idx].astype(np.float32)
        next_state = self.state[nxt].astype(np.float32)
        action = np.zeros((B, NUM_ACTIONS, 1, 1), np.float32)
        action[np.arange(B), self.action[nxt]] = 1
        reward = self.reward[nxt].astype(np.float32).reshape(B, 1, 1, 1)
        nonterm = self.non_terminal[nxt].astype(np.float32).reshape(B, 1, 1, 1)
        return state, action, reward, next_state, nonterm


def draw_indices(rng, valid, head, B):
    """Index draw of replay.py:147-159 (uniform subset without replacement,
    redraw while head-1 is in it, sorted), on a numpy Generator."""
    if B >= valid:
        raise ValueError("Can't draw sample of size %d from replay dataset of size %d"
                         % (B, valid))
    while True:
        idx = rng.choice(valid, size=B, replace=False)
        if (head - 1) not in idx:
            return np.sort(idx)


# --------------------------------------------------------------------------
# param-server apply rules (server.py:49-124) on flat float32 buffers
# --------------------------------------------------------------------------
def sgd_update(theta, g, lr):
    """server.py:81-83 -> apply_descent with scale=None (:66-68)."""
    return (theta - np.float32(lr) * g).astype(np.float32)


def rmsprop_update(theta, g, cache, lr, decay=0.9):
    """server.py:86-105.  First call: cache = g^2 and the update uses it.
    Later calls: the update uses the PREVIOUS cache (d_rmsprop is copied
    before the cache is refreshed), then cache = decay*c + (1-decay)*g^2."""
    g = g.astype(np.float32)
    if cache is None:
        c_use = g * g
        new_cache = c_use
    else:
        c_use = cache
        new_cache = (np.float32(decay) * cache + np.float32(1 - decay) * (g * g)).astype(np.float32)
    th = theta - np.float32(lr) * g / np.sqrt(c_use + np.float32(EPS))
    return th.astype(np.float32), new_cache.astype(np.float32)


def adagrad_update(theta, g, acc, lr):
    """server.py:108-124: G = g^2 (first) or G += g^2, update with CURRENT G."""
    g = g.astype(np.float32)
    acc = g * g if acc is None else (acc + g * g)
    th = theta - np.float32(lr) * g / np.sqrt(acc + np.float32(EPS))
    return th.astype(np.float32), acc.astype(np.float32)


def momentum_caffe_update(theta, g, v, lr_mult, wd_mult, base_lr=0.01, momentum=0.9,
                          weight_decay=0.0005):
    """Caffe SGDSolver::ComputeUpdateValue with solver.prototxt:4-11 values
    (not the reference's distributed rule; optional, "solver.prototxt
    semantics"): v = m*v + lr*(g + wd*theta); theta -= v.  Per-element lr/wd
    multipliers come from blobs_lr {1,2} and weight_decay {1,0}."""
    lr = np.float32(base_lr) * lr_mult
    wd = np.float32(weight_decay) * wd_mult
    v = (np.float32(momentum) * v + lr * (g + wd * theta)).astype(np.float32)
    return (theta - v).astype(np.float32), v


def special_update(model):
    """server.py:127-137: copy every Q* blob to P*."""
    for key in list(model.keys()):
        if key[0] == "Q":
            model["P" + key[1:]] = model[key]
    return model


# --------------------------------------------------------------------------
# messaging byte layout (barista/messaging.py)
# --------------------------------------------------------------------------
def create_message_ref(params, iteration):
    """messaging.py:13-40: pack('ii', iter, hlen) + pickle(header) + raw fp32."""
    meta = collections.OrderedDict()
    data = b""
    for name in params:
        meta[name] = [tuple(b.shape) for b in params[name]]
        for b in params[name]:
            data += np.ascontiguousarray(b, np.float32).tobytes()
    header = pickle.dumps(meta, 2)
    return struct.pack("ii", iteration, len(header)) + header + data


def load_gradient_message_ref(msg):
    """messaging.py:128-164."""
    (hlen,) = struct.unpack("i", msg[:4])
    header = pickle.loads(msg[4:4 + hlen])
    data = msg[4 + hlen:]
    idx = 0
    grads = {}
    for name in header:
        grads[name] = []
        for shape in header[name]:
            n = int(np.prod(shape)) * 4
            grads[name].append(np.frombuffer(data[idx:idx + n], np.float32).reshape(shape))
            idx += n
    return grads


def epsilon(iter_num, frame_limit=50000, emax=1.0, emin=0.1):
    """expgain.py:55-60 linear epsilon schedule."""
    if iter_num > frame_limit:
        return emin
    return emin + (emax - emin) * max(frame_limit - iter_num, 0) / frame_limit
