"""Native dispatch under MPPI_AQL_FENCES (diagnostic packet fence scopes): C3 step rate of
back-to-back batches and bit-exactness of u_prev / costs against HIP dispatch (tools/)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
ST = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, np.float64)


def mk(mode):
    os.environ["MPPI_DISPATCH"] = mode
    e = Engine(make_config("arm", device=0, seed=3, n_samples=4096, n_horizon=32, state_f64=True))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(ST)
    return e


h, a = mk("hip"), mk("aql")
for e in (h, a):
    e.run_steps(300)
    e.synchronize()
ok = np.array_equal(h.get_u_prev(), a.get_u_prev()) and np.array_equal(h.get_costs(), a.get_costs())
rates = []
for _ in range(5):
    a.run_steps(50)
    a.synchronize()
    t0 = time.perf_counter()
    a.run_steps(1000)
    a.synchronize()
    rates.append((time.perf_counter() - t0) / 1000 * 1e6)
print(f"fences={os.environ.get('MPPI_AQL_FENCES', 'default 0000')} bit-exact vs HIP after 300 steps: {ok}  "
      f"us/step (1000-step batches): median {np.median(rates):.2f}  all {[round(x, 2) for x in rates]}")
