"""Keep-alive (mppi_set_keepalive): a host thread of the engine launches a one-wave kernel on its
own stream while the controller idles between ticks (the node's rospy.Rate(100) loop,
kinova.py:101).  It must touch no engine state -- the control calls return bit for bit what an
engine without it returns -- launch while idle, stop when turned off, reject bad periods, and
be stopped by mppi_destroy."""
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


def test_keepalive_changes_no_result_and_stops():
    from quadrotor_manipulator_mppi_amd._capi import MPPIError
    plain, kept = _engine(), _engine()
    assert kept.keepalive() == (0, 0)
    kept.set_keepalive(200)
    rng = np.random.default_rng(0)
    for i in range(30):
        st = STATE.copy()
        st[7:14] += rng.normal(0.0, 0.01, 7)
        o1, u1, s1 = plain.step(st)
        o2, u2, s2 = kept.step(st)
        assert np.array_equal(o1, o2) and np.array_equal(u1, u2), f"call {i}: the keep-alive changed a result"
        assert s1[0].rho == s2[0].rho
        time.sleep(0.002 if i % 3 else 0.01)   # idle gaps: the keep-alive launches in them
    kept.run_steps(20)
    plain.run_steps(20)
    kept.synchronize()
    plain.synchronize()
    assert np.array_equal(kept.get_u_prev(), plain.get_u_prev())
    period, n = kept.keepalive()
    assert period == 200 and n > 0, (period, n)
    kept.set_keepalive(0)
    _, n_off = kept.keepalive()
    time.sleep(0.02)
    assert kept.keepalive() == (0, n_off), "no launches after it was turned off"
    for bad in (-1, 50, 2_000_000):
        with pytest.raises(MPPIError):
            kept.set_keepalive(bad)
    kept.set_keepalive(1000)   # left on: close() (mppi_destroy) stops the thread
    time.sleep(0.005)
    kept.close()
    plain.close()
