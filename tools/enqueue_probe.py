"""Host enqueue time of mppi_run_steps per control step vs the synchronized step time (tools/, not shipped)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
for model, K, H, f64 in (("arm", 4096, 32, True), ("wholebody", 8192, 64, False)):
    e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=f64))
    sd = [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * (7 if model == "arm" else 10)
    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5]); e.set_state(np.array(sd, np.float64))
    e.run_steps(100); e.synchronize()
    for n in (200, 2000):
        t0 = time.perf_counter(); e.run_steps(n); t1 = time.perf_counter(); e.synchronize(); t2 = time.perf_counter()
        print(f"{model} n={n}: host enqueue {1e6*(t1-t0)/n:.2f} us/step, total {1e6*(t2-t0)/n:.2f} us/step", flush=True)
    e.close()
