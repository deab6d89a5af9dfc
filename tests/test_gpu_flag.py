"""The completion-flag protocol under stress (mppi_finalize.hip tail): the host reads a
step's outputs as soon as every (vehicle, dim) flag carries the step's sequence number, so
the flag must never become visible before the outputs it guards.  Thousands of control
calls with a changing state and target: the outputs read behind the flags must equal a
second read of the same buffer after a full stream synchronize, call by call, and follow
the reference update (qdes from the OLD u_prev[0], mppi.py:157)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]


def _engine(model, **kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    return Engine(make_config(model, device=0, **kw))


@pytest.mark.parametrize("model,K,H", [("arm", 1024, 32), ("drone", 512, 32), ("wholebody", 1024, 64)])
def test_outputs_visible_with_their_flags(model, K, H):
    e = _engine(model, n_samples=K, n_horizon=H, seed=7)
    rng = np.random.default_rng(1)
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    if model == "arm":
        base = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7)
    elif model == "drone":
        base = np.array([0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
    else:
        base = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 10)
    n = int(os.environ.get("MPPI_FLAG_STRESS_N", "1500"))
    mismatches = 0
    for i in range(n):
        state = base.copy()
        state[:3] += rng.normal(0, 0.05, 3)
        if model != "drone":
            state[7:14] += rng.normal(0, 0.05, 7)
        out1, u01, st1 = e.step(state)
        e.synchronize()
        out2, u02, st2 = e.read_outputs()
        if not (np.array_equal(out1, out2) and np.array_equal(u01, u02) and st1[0].rho == st2[0].rho):
            mismatches += 1
        if model == "drone" and i % 100 == 0:   # drone_mppi.py:168-169 from the step's own u0
            x0, v0 = state[:3].astype(np.float32), state[3:6].astype(np.float32)
            np.testing.assert_allclose(out1[0, :3], x0 + v0 * np.float32(0.01) + 0.5 * u01[0] * np.float32(1e-4),
                                       rtol=1e-5, atol=1e-5)
    e.close()
    assert mismatches == 0, f"{mismatches} of {n} calls read outputs the flags did not cover"
