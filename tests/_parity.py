"""Shared fp32-vs-float64 comparison for the GPU parity tests.

north_star: "Q-values, targets, gradients and post-update weights must match
within fp32 rtol 1e-4".  Two elementwise rules, neither with a tensor-wide
absolute floor:

* blobs and gradients (``close(..., mag=M)``, ``check_full_pass``): every
  element within  rtol * |ref| + COND * M,  rtol = 1e-4, COND = 2e-7, where M
  is the oracle's per-element sum of |terms| (``oracle.ref_numpy.magnitudes``:
  the same computation on absolute values).  Where the terms do not cancel
  this is rtol 1e-4; where they do (a Q_out of 0.011 summed from 512 products
  of size ~2.5) the element may move by the fp32 rounding of its own terms --
  COND = 2e-7 is ~3.4 fp32 ulps of M, 6x the worst measured (3.2e-8 * M).
* parameters and optimizer state (no cancellation structure): rtol 1e-4 for
  every element with |ref| >= 1e-3 of the tensor's max, and an absolute 1e-6
  of that max (~16 ulps of the largest element) below it.

NaN / inf count as mismatches.  The maximum relative error over the well-
conditioned elements is returned (and printed) so logs show how close each
tensor is.
"""
import numpy as np

RTOL = 1e-4
FLOOR = 1e-3
ATOL = 1e-6
COND = 2e-7     # fp32 rounding allowance per unit of |terms| (~3.4 ulps; measured max 3.2e-8)


def close(gpu, ref, rtol=RTOL, what="", floor=FLOOR, atol=ATOL, quiet=False, mag=None,
          cond=COND):
    """mag (the oracle's magnitudes(): per-element sum of |terms|): every
    element is bounded by rtol * |ref| + cond * mag -- relative where the
    terms do not cancel, fp32 rounding of its own terms where they do; no
    tensor-wide floor.  Without mag: the floor rule of the module docstring."""
    gpu = np.asarray(gpu, np.float64)
    ref = np.asarray(ref, np.float64)
    assert gpu.shape == ref.shape or gpu.size == ref.size, (what, gpu.shape, ref.shape)
    gpu = gpu.reshape(ref.shape)
    if ref.size == 0:
        return 0.0
    scale = float(np.max(np.abs(ref)))
    err = np.abs(gpu - ref)
    if mag is not None:
        m = np.asarray(mag, np.float64).reshape(ref.shape)
        tol = rtol * np.abs(ref) + cond * m + 1e-30
        big = (np.abs(ref) >= 0.1 * m) & (ref != 0)   # well-conditioned (< 10x cancellation)
    else:
        big = np.abs(ref) >= floor * scale
        tol = np.where(big, rtol * np.abs(ref), atol * scale) + 1e-30
    bad = ~(err <= tol)
    max_rel = float(np.max(err[big] / np.abs(ref[big]))) if big.any() else 0.0
    if not quiet:
        if mag is not None:
            cm = float(np.max(err / (np.asarray(mag, np.float64).reshape(ref.shape) + 1e-300)))
            print("%-28s max rel err %.3g (%d/%d well-conditioned), max err/|terms| %.3g"
                  % (what, max_rel, int(big.sum()), ref.size, cm))
        else:
            small_abs = float(np.max(err[~big]) / scale) if (~big).any() and scale > 0 else 0.0
            print("%-28s max rel err %.3g (%d/%d elements >= %.0e of scale %.3g), below: max "
                  "abs err %.3g of scale" % (what, max_rel, int(big.sum()), ref.size, floor,
                                             scale, small_abs))
    if bad.any():
        i = np.unravel_index(np.argmax(np.where(bad, err / tol, 0)), ref.shape)
        raise AssertionError("%s: %d/%d elements off (%s); worst at %s: gpu %.9g ref %.9g%s" % (
            what, int(bad.sum()), bad.size,
            "rtol %g + %g * |terms|" % (rtol, cond) if mag is not None else
            "rtol %g above %g of scale %.3g, atol %g of scale below" % (rtol, floor, scale, atol),
            i, gpu[i], ref[i], "" if mag is None else " |terms| %.3g" % np.asarray(mag).reshape(
                ref.shape)[i]))
    return max_rel


def fc4_near_ties(ref, net, cache, grads, blobs, pQ, mb, g_gpu=None, tie4=COND, max_frac=1e-4):
    """fc4's ReLU (train_val.prototxt:186-191) at a genuine fp32-vs-fp64
    near-tie: a unit (b, n) whose float64 pre-activation lies within tie4 of
    its own sum of |terms| (COND: the fp32 rounding bound of the blobs) of 0
    may be live on the GPU and dead in the oracle
    (or the reverse).  Its side is read off the GPU's fc4 bias gradient
    (db4[n] = sum_b dh4[b][n]: that unit's dh4 is in it or not -- the two
    candidates differ by |dQ . W5[:, n]|, far above fp32 rounding) and adopted
    for that unit only.  Returns (h4 mask or None, adopted count)."""
    pre4, flat = cache["pre4"], cache["flat"]
    W4 = np.asarray(pQ["Qfc4"][0], np.float64).reshape(512, -1)
    b4 = np.asarray(pQ["Qfc4"][1], np.float64).reshape(-1)
    m4 = np.abs(flat) @ np.abs(W4).T + np.abs(b4)
    near = np.argwhere((np.abs(pre4) <= tie4 * m4) & (m4 > 0))   # (exact zeros agree)
    if len(near) == 0:
        return None, 0
    assert len(near) <= max(4, max_frac * pre4.size), ("too many fc4 near-ties", len(near))
    if g_gpu is None:
        g_gpu = net.get_grads_flat()
    db4_gpu = np.asarray(net.split(g_gpu, "Q")["Qfc4"][1], np.float64).reshape(-1)
    db4_ref = np.asarray(grads["Qfc4"][1], np.float64).reshape(-1)
    B = pre4.shape[0]
    act = np.asarray(mb[1], np.float64).reshape(B, 4)
    dq = act * ((blobs["Q_sa"] - blobs["target_Q_sa"]) / B)[:, None]
    W5 = np.asarray(pQ["Q_out"][0], np.float64).reshape(4, 512)
    full = dq @ W5                                   # dh4 before the ReLU mask
    mask = pre4 > 0
    adopted = 0
    for (b, n) in near:
        d = full[b, n] * (-1.0 if mask[b, n] else 1.0)   # what flipping does to db4[n]
        if abs(db4_gpu[n] - (db4_ref[n] + d)) < abs(db4_gpu[n] - db4_ref[n]):
            mask[b, n] = not mask[b, n]
            db4_ref = db4_ref.copy()
            db4_ref[n] += d
            adopted += 1
    return (mask if adopted else None), adopted


def full_pass_gpu_routing(ref, net, pQ, pP, mb, max_frac=1e-4, tie=2e-5, g_gpu=None,
                          with_mask=False):
    """The oracle's full pass on minibatch ``mb`` with max-pool routing taken
    from the GPU's last forward (``net.pool_mask``) wherever the two differ --
    and only there, after proving every difference is a genuine fp32-vs-fp64
    near-tie: both candidate values (or the max vs 0 for a ReLU'd window)
    agree to ``tie`` of the layer's activation scale, and at most ``max_frac``
    of the windows differ -- and fc4's ReLU mask likewise at proven near-ties
    (fc4_near_ties).  Returns (blobs, grads, n_ties) (+ the fc4 mask with
    with_mask)."""
    blobs, grads, cache = ref.full_pass(pQ, pP, *mb, return_cache=True)
    routes, nties = {}, 0
    for i in (1, 2, 3):
        g_code = net.pool_mask(i)
        r_code = ref.route_codes(cache["act%d" % i], cache["arg%d" % i])
        a = cache["act%d" % i]
        Bn, C, H, W = a.shape
        win = a.reshape(Bn, C, H // 2, 2, W // 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(
            Bn, C, H // 2, W // 2, 4)
        scale = a.max()
        dis = np.argwhere(g_code != r_code)
        assert len(dis) <= max(2, max_frac * g_code.size), ("too many routing differences", i,
                                                            len(dis))
        for (b, c, y, x) in dis:
            w = win[b, c, y, x]
            vals = [w[k] if k < 4 else 0.0 for k in (g_code[b, c, y, x], r_code[b, c, y, x])]
            assert abs(vals[0] - vals[1]) <= tie * scale, ("non-tie routing mismatch", i, w)
        nties += len(dis)
        routes[i] = g_code
    if nties:
        blobs, grads = ref.full_pass(pQ, pP, *mb, routes=routes)
    h4_mask, n4 = fc4_near_ties(ref, net, cache, grads, blobs, pQ, mb, g_gpu)
    if n4:
        blobs, grads = ref.full_pass(pQ, pP, *mb, routes=routes, h4_mask=h4_mask)
        nties += n4
    if with_mask:
        return blobs, grads, nties, h4_mask
    return blobs, grads, nties


def check_full_pass(ref, net, pQ, pP, mb, grads_gpu=None, quiet=False, what=""):
    """Blobs and Q gradients of the GPU's last forward/backward on ``mb``
    against the oracle (GPU routing at proven near-ties), each element within
    rtol 1e-4 + COND (2e-7) * (its sum of |terms|).  Returns the near-tie count."""
    blobs, grads, nties, h4_mask = full_pass_gpu_routing(ref, net, pQ, pP, mb, g_gpu=grads_gpu,
                                                         with_mask=True)
    routes = {i: net.pool_mask(i) for i in (1, 2, 3)}
    mblobs, mgrads = ref.magnitudes(pQ, pP, *mb, routes=routes, h4_mask=h4_mask)
    B = net.batch
    for name, shape in (("Q_out", (B, 4)), ("P_out", (B, 4)), ("Q_sa", (B,)), ("P_sa", (B,)),
                        ("target_Q_sa", (B,))):
        close(net.blob(name).reshape(shape), blobs[name], what=what + name, mag=mblobs[name],
              quiet=quiet)
    close(float(net.blob("loss")), blobs["loss"], what=what + "loss", mag=mblobs["loss"],
          quiet=quiet)
    g = net.split(net.get_grads_flat() if grads_gpu is None else grads_gpu, "Q")
    for name in grads:
        for i in range(2):
            close(g[name][i], grads[name][i], what="%s%s[%d]" % (what, name, i),
                  mag=mgrads[name][i], quiet=quiet)
    return blobs, grads, nties
