"""Control-step rate of back-to-back mppi_run_steps (wall clock), with and without
trajectory stores:  python tools/step_rate.py arm 4096 32"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
model, K, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "drone": [0, 0, 1, 0, 0, 0], "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
for traj in (True, False):
    e = Engine(make_config(model, n_samples=K, n_horizon=H, store_trajectory=traj, state_f64=(model == "arm")))
    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(np.array(sd, np.float64))
    e.run_steps(100); e.synchronize()
    n = 2000
    t0 = time.perf_counter(); e.run_steps(n); e.synchronize(); dt = time.perf_counter() - t0
    t0 = time.perf_counter(); e.run_steps(300); t_enq = time.perf_counter() - t0; e.synchronize()
    r, f = e.kernel_timing(200)
    print(f"{os.path.basename(os.environ.get('MPPI_HIP_LIB', 'default'))} {model} K={K} H={H} traj={traj}: "
          f"{dt / n * 1e6:7.2f} us/step, host enqueue {t_enq / 300 * 1e6:6.2f} us/step  (rollout {r:6.2f} us, finalize {f:6.2f} us back-to-back)", flush=True)
    e.close()
