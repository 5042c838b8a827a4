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


def full_pass_gpu_routing(ref, net, pQ, pP, mb, max_frac=1e-4, tie=2e-5):
    """The oracle's full pass on minibatch ``mb`` with max-pool routing taken
    from the GPU's last forward (``net.pool_mask``) wherever the two differ --
    and only there, after proving every difference is a genuine fp32-vs-fp64
    near-tie: both candidate values (or the max vs 0 for a ReLU'd window)
    agree to ``tie`` of the layer's activation scale, and at most ``max_frac``
    of the windows differ.  Returns (blobs, grads, n_ties)."""
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
    return blobs, grads, nties


def check_full_pass(ref, net, pQ, pP, mb, grads_gpu=None, quiet=False, what=""):
    """Blobs and Q gradients of the GPU's last forward/backward on ``mb``
    against the oracle (GPU routing at proven near-ties), each element within
    rtol 1e-4 + COND (2e-7) * (its sum of |terms|).  Returns the near-tie count."""
    blobs, grads, nties = full_pass_gpu_routing(ref, net, pQ, pP, mb)
    routes = {i: net.pool_mask(i) for i in (1, 2, 3)}
    mblobs, mgrads = ref.magnitudes(pQ, pP, *mb, routes=routes)
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
