"""deepq16's four-launch step (csrc/small.h, csrc/small_bwd.h): which ctxs run
it, and what happens when one of its inter-workgroup meetings fails.

K1, K2 and K4 hand data between workgroups of one launch through a spin
meeting (small.h ``meet``).  That is only safe when every meeting workgroup is
resident at once, so ``ddq_create`` checks it with the occupancy API and runs
the general kernels otherwise (``ddq_small_path``).  Should a meeting still
fail (a party never arrives), the spin gives up after a bound instead of
hanging, the launches write no parameter, optimizer state, P copy or
iteration, and ``ddq_synchronize`` returns DDQ_ESTATE, after which the ctx
steps on from its last good update.  ``ddq_inject_fault(DDQ_FAULT_MEET_TIMEOUT)``
launches the next eager step's fc4 chain one workgroup short to drive exactly
that path.
"""
import numpy as np
import pytest

from _parity import check_full_pass, close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ddq():
    import ddq as m
    return m


@pytest.fixture(scope="module")
def ref():
    from oracle import ref_numpy
    return ref_numpy


@pytest.mark.parametrize("S,B,on,why", [(16, 1, True, ""), (16, 32, True, ""),
                                        (16, 256, True, ""), (16, 300, False, "batch > 256"),
                                        (64, 32, False, "frame != 16")])
def test_small_path_selection(ddq, S, B, on, why):
    net = ddq.DeepQNet(batch=B, frame=S)
    got, reason = net.small_path()
    assert got == on, reason
    assert reason == why
    net.close()


def test_fault_needs_the_small_path(ddq):
    net = ddq.DeepQNet(batch=32, frame=24)
    with pytest.raises(ddq._lib.DDQError) as ei:
        net.inject_fault("meet_timeout")
    assert ei.value.code == ddq._lib.DDQ_ESTATE
    net.inject_fault(None)   # disarming is always fine
    net.close()


def test_meet_timeout_reports_and_applies_nothing(ddq, ref):
    from ddq.expgain import synthetic_transitions
    from ddq.params import init_params_flat
    S, B, N, lr = 16, 32, 512, 1e-4
    st, ac, rw, nt = synthetic_transitions(N, S, seed=5)
    theta = init_params_flat(S, seed=42)
    net = ddq.DeepQNet(batch=B, frame=S)
    assert net.small_path()[0]
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    net.replay_create(N)
    net.replay_import(st, ac, rw, nt.astype(np.uint8), 0, N)
    cfg = net.step_cfg("rmsprop", lr=lr, target_period=10, seed=3)
    for _ in range(3):
        net.step(cfg)
    net.synchronize()
    q0, p0, s0 = net.get_flat(0), net.get_flat(1), net.optimizer_state()
    draws = net.replay_draws()

    net.inject_fault("meet_timeout")
    net.step(cfg)                                    # K2 launched one workgroup short
    with pytest.raises(ddq._lib.DDQError) as ei:
        net.synchronize()
    assert ei.value.code == ddq._lib.DDQ_ESTATE
    assert "fc4 chain fan-in" in ei.value.msg
    # nothing of the failed step reached the model
    np.testing.assert_array_equal(net.get_flat(0), q0)
    np.testing.assert_array_equal(net.get_flat(1), p0)
    np.testing.assert_array_equal(net.optimizer_state(), s0)
    assert net.replay_draws() == draws + 1           # (its minibatch was drawn)
    net.synchronize()                                # the flag was cleared

    # the ctx steps on from the last good update: the next step against the
    # oracle's step from (q0, p0, s0) on the minibatch it drew
    net.step(cfg)
    net.synchronize()
    idx = net.read_indices()
    r = ref.ReplayRef((4, S, S), N)
    r.state, r.action, r.reward, r.non_terminal = st, ac, rw, np.asarray(nt).astype(bool)
    r.head, r.valid = 0, N
    _, grads, _ = check_full_pass(ref, net, ref.unflatten(q0, S, "Q"), ref.unflatten(p0, S, "P"),
                                  r.gather(idx), what="after recovery ")
    g = ref.flatten(grads).astype(np.float32)
    th_ref, st_ref = ref.rmsprop_update(q0, g, s0, lr, 0.9)
    close(net.get_flat(0), th_ref, what="theta_Q after recovery")
    close(net.optimizer_state(), st_ref, what="cache after recovery")
    np.testing.assert_array_equal(net.get_flat(1), p0)   # 4 updates: no P <- Q yet
    # pipelined graphs after it, across the P <- Q sync at 10
    net.step_pipelined(cfg, 12)
    net.synchronize()
    q1, p1 = net.get_flat(0), net.get_flat(1)
    assert np.isfinite(q1).all() and not np.array_equal(q1, q0) and not np.array_equal(p1, p0)
    net.close()
