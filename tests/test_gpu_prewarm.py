"""Prewarm (mppi_set_prewarm): a host thread of the engine predicts the next control call from the
cadence of the last ones and touches the engine's native queue (pairs of one-wave packets into a
scratch word) through a window before it -- for the node's rospy.Rate(100) loop (kinova.py:101).
It must change no result: control calls and later batches (whose step word is re-uploaded because
the touches moved the queue's packet indices) return bit for bit what an engine without it returns.
It must touch at a steady cadence, stop when turned off, reject bad windows, and be stopped by
mppi_destroy."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
STATE = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, np.float64)


def _engine():
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    e = Engine(make_config("arm", device=0, n_samples=512, n_horizon=32, state_f64=True, seed=5))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(STATE)
    return e


def test_prewarm_changes_no_result_and_stops():
    from quadrotor_manipulator_mppi_amd._capi import MPPIError
    plain, warm = _engine(), _engine()
    assert warm.prewarm() == (0, 0)
    warm.set_prewarm(200)
    rng = np.random.default_rng(0)
    period = 0.003
    nxt = time.perf_counter()
    for i in range(40):   # calls on a 3 ms tick, as rospy.Rate.sleep spaces them
        st = STATE.copy()
        st[7:14] += rng.normal(0.0, 0.01, 7)
        o1, u1, s1 = plain.step(st)
        o2, u2, s2 = warm.step(st)
        assert np.array_equal(o1, o2) and np.array_equal(u1, u2), f"call {i}: the prewarm changed a result"
        assert s1[0].rho == s2[0].rho
        nxt += period
        time.sleep(max(0.0, nxt - time.perf_counter()))
    window, touches = warm.prewarm()
    assert window == 200 and touches > 0, (window, touches)
    for _ in range(3):   # batches after touches: the step word follows the moved packet indices
        warm.run_steps(20)
        plain.run_steps(20)
        warm.synchronize()
        plain.synchronize()
        assert np.array_equal(warm.get_u_prev(), plain.get_u_prev())
        o1, u1, _ = plain.step(STATE)
        o2, u2, _ = warm.step(STATE)
        assert np.array_equal(o1, o2) and np.array_equal(u1, u2)
        time.sleep(period)
    # batches issued inside the touch window (100 us before the predicted call): touches land
    # between and around them; each batch's rollouts must still run the steps prepared for them
    nxt = time.perf_counter()
    for i in range(30):
        o1, u1, _ = plain.step(STATE)
        o2, u2, _ = warm.step(STATE)
        assert np.array_equal(o1, o2) and np.array_equal(u1, u2), f"window call {i}"
        nxt += period
        time.sleep(max(0.0, nxt - 0.0001 - time.perf_counter()))
        warm.run_steps(2)
        plain.run_steps(2)
    warm.synchronize()
    plain.synchronize()
    assert np.array_equal(warm.get_u_prev(), plain.get_u_prev())
    warm.set_prewarm(0)
    _, t_off = warm.prewarm()
    for _ in range(10):
        warm.step(STATE)
        time.sleep(period)
    assert warm.prewarm() == (0, t_off), "no touches after it was turned off"
    for bad in (-1, 20, 6000):
        with pytest.raises(MPPIError):
            warm.set_prewarm(bad)
    warm.set_prewarm(100)   # left on: close() (mppi_destroy) stops the thread
    for _ in range(8):
        warm.step(STATE)
        time.sleep(0.002)
    warm.close()
    plain.close()


def test_dropin_prewarm_option_changes_nothing():
    """The drop-in arm class with ``prewarm_us`` (the node's 100 Hz loop, kinova.py:101-116) returns
    what the class without it returns, and its engine touches its queue between the ticks."""
    import torch
    from quadrotor_manipulator_mppi_amd.mppi_solver.mppi import MPPI
    q = torch.tensor([0, 0, 1, 0, 0, 0, 1] + HOME, dtype=torch.float64)
    v = torch.zeros(13, dtype=torch.float64)
    plain, warm = MPPI(n_samples=256, verbose=False), MPPI(n_samples=256, verbose=False, prewarm_us=200)
    nxt = time.perf_counter()
    for i in range(30):
        for m in (plain, warm):
            m.update_joint(q, v)
        q1, v1 = plain.compute_control_input()
        q2, v2 = warm.compute_control_input()
        assert torch.equal(torch.as_tensor(q1), torch.as_tensor(q2)) and torch.equal(torch.as_tensor(v1), torch.as_tensor(v2)), i
        nxt += 0.003
        time.sleep(max(0.0, nxt - time.perf_counter()))
    assert warm._engine.prewarm()[0] == 200 and warm._engine.prewarm()[1] > 0
    assert plain._engine.prewarm() == (0, 0)
