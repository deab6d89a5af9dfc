"""Native vs HIP dispatch, step by step (tools/, diagnostics): where do they part?"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
ST = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, np.float64)


def mk(mode, K=1024):
    os.environ["MPPI_DISPATCH"] = mode
    e = Engine(make_config("arm", device=0, seed=11, n_samples=K, n_horizon=32))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(ST)
    return e


def cmp(tag, h, a):
    h.synchronize(); a.synchronize()
    ch, ca = h.get_costs(), a.get_costs()
    uh, ua = h.get_u_prev(), a.get_u_prev()
    print(f"{tag}: dispatch={a.dispatch_info()!r} costs equal={np.array_equal(ch, ca)} "
          f"(max|d|={np.abs(ch - ca).max():.3g}) u_prev equal={np.array_equal(uh, ua)} (max|d|={np.abs(uh - ua).max():.3g})")
    return np.array_equal(ch, ca)


h, a = mk("hip"), mk("aql")
for i in range(4):
    h.run_steps(1); a.run_steps(1)
    cmp(f"after batch {i + 1} of 1 step", h, a)
# which step counter did the native engine's last rollout use?  replay on a HIP engine
a2 = mk("aql")
a2.run_steps(1); a2.synchronize()
c_a = a2.get_costs()
for ctr in range(0, 3):
    h2 = mk("hip")
    h2.set_step_counter(ctr)
    h2.run_steps(1); h2.synchronize()
    print("native 1-step costs == hip step_ctr", ctr, ":", np.array_equal(h2.get_costs(), c_a))
    h2.close()
