"""Tick-by-tick check of the asynchronous param server (DDQ_EXCHANGE_ASYNC)
against param-server/server.py replayed in the same arrival order.

server.py:196-209 applies every pushed gradient on arrival (apply_descent,
:49-78, with the rule's state carried from push to push) and :181-193 copies
Q -> P on a pull that sees iteration % special_update_period == 0.  A worker
(main.py:61-112) pushes the gradient it computed on the model it last pulled,
pulls, and computes its next gradient there.

The group runs ONE tick at a time (ddq_group_async_ticks), so every quantity
of the tick is observable:
  before tick t (worker w):  g = w's gradient buffer (the push), the central
                             model = the last puller's replica, the owners'
                             optimizer-state shards;
  after it:                  w's replica == apply(central, g, state) (server
                             rule, teacher-forced on the GPU's own inputs),
                             the owners' state likewise, w's P == the central
                             P iff a special update happened since its last
                             pull (else unchanged), and w's NEW gradient ==
                             the oracle at (its pulled Q and P, its next
                             minibatch draw) -- tests/_parity.py tolerances.
"""
import numpy as np

from _parity import check_full_pass, close


def apply_ref(ref, rule, theta, g, state, lr):
    if rule == "sgd":
        return ref.sgd_update(theta, g, lr), None
    if rule == "rmsprop":
        return ref.rmsprop_update(theta, g, state, lr)
    return ref.adagrad_update(theta, g, state, lr)


def owner_state(nets):
    """Optimizer state as the owners hold it (shard r on member r,
    L = ceil(P / (64 W)) * 64, api.hip setup_shards)."""
    P = nets[0].num_params
    L = -(-P // (64 * len(nets))) * 64
    out = np.empty(P, np.float32)
    for r, n in enumerate(nets):
        out[r * L:(r + 1) * L] = n.optimizer_state()[r * L:(r + 1) * L]
    return out


def run_checked(ddq, ref, nets, arr, cfg, order, minibatch, rule, lr, period, theta0,
                grad_check=lambda t, w: True, what=""):
    """Run `order` tick by tick on the group; minibatch(w, d) -> the oracle's
    inputs of member w's d-th device draw (its index log)."""
    W = len(nets)
    S = nets[0].frame
    ddq.DeepQNet.group_async_ticks(nets, cfg, [], arr)      # begin: first gradients
    draws = [0] * W
    for w, n in enumerate(nets):
        if grad_check(-1, w):
            check_full_pass(ref, n, ref.unflatten(theta0, S, "Q"), ref.unflatten(theta0, S, "P"),
                            minibatch(w, 0), quiet=True, what="%sinit w%d " % (what, w))
    central, pc, it = theta0.copy(), theta0.copy(), 0
    state = None
    last_pull = [0] * W
    for t, w in enumerate(order):
        g = nets[w].get_grads_flat()
        prev_p = nets[w].get_flat(1)
        ddq.DeepQNet.group_async_ticks(nets, cfg, [w], arr)
        want, want_state = apply_ref(ref, rule, central, g, state, lr)
        got = nets[w].get_flat(0)
        close(got, want, what="%stick %d w%d central" % (what, t, w), quiet=True)
        it += 1
        if period and it % period == 0:
            pc = got.copy()
        pull_p = bool(period) and it // period > last_pull[w] // period
        last_pull[w] = it
        gp = nets[w].get_flat(1)
        if pull_p:
            np.testing.assert_array_equal(gp, pc)
        else:
            np.testing.assert_array_equal(gp, prev_p)
        if want_state is not None:
            ost = owner_state(nets)
            close(ost, np.asarray(want_state, np.float32),
                  what="%stick %d opt state" % (what, t), quiet=True)
            state = ost                    # teacher forcing: the owners' own state
        central = got                      # ... and the GPU's central model
        draws[w] += 1
        if grad_check(t, w):
            check_full_pass(ref, nets[w], ref.unflatten(got, S, "Q"), ref.unflatten(gp, S, "P"),
                            minibatch(w, draws[w]), quiet=True,
                            what="%stick %d w%d grad " % (what, t, w))
    return central
