"""Rollout / finalize kernel time by three methods (arm C3 by default):
(1) mppi_kernel_timing: one event pair around n back-to-back launches of ONE kernel;
(2) per-launch event pairs inside the real step sequence (mppi_enable_timing);
(3) step time of back-to-back steps (mppi_run_steps) for reference.
   python tools/timing_probe.py [model K H]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

model = sys.argv[1] if len(sys.argv) > 1 else "arm"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
H = int(sys.argv[3]) if len(sys.argv) > 3 else 32
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=(model == "arm")))
e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
e.set_state(np.array(sd, np.float64))
e.run_steps(100); e.synchronize()
r1, f1 = e.kernel_timing(500)
e.enable_timing(True)
e.run_steps(500); e.synchronize()
t = e.timing()
e.enable_timing(False)
r2, f2 = 1e3 * t["rollout_ms_total"] / t["n_rollout"], 1e3 * t["finalize_ms_total"] / t["n_finalize"]
n = 2000
t0 = time.perf_counter(); e.run_steps(n); e.synchronize(); st = (time.perf_counter() - t0) / n * 1e6
print(f"{model} K={K} H={H}: back-to-back single-kernel events rollout {r1:.2f} us finalize {f1:.2f} us | "
      f"per-launch events in sequence rollout {r2:.2f} us finalize {f2:.2f} us | step {st:.2f} us")
