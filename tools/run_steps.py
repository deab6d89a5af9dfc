"""n back-to-back control steps of one engine (for rocprofv3 kernel traces):
   python tools/run_steps.py arm 4096 32 [n]"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
model, K, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 500
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "drone": [0, 0, 1, 0, 0, 0], "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=(model == "arm")))
e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
e.set_state(np.array(sd, np.float64))
e.run_steps(50); e.synchronize()
t0 = time.perf_counter(); e.run_steps(n); e.synchronize(); dt = time.perf_counter() - t0
print(f"{model} K={K} H={H}: {dt / n * 1e6:.2f} us/step", flush=True)
