"""Per-phase wave timelines of the rollout / finalize kernels (stamps build).
   MPPI_HIP_LIB=.../libmppi_hip_stamps.so MPPI_STAMPS=1 python tools/stamp_probe.py drone 256 32"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
model, K, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
bt = int(sys.argv[4]) if len(sys.argv) > 4 else 0
e = Engine(make_config(model, n_samples=K, n_horizon=H, block_threads=bt, state_f64=(model == "arm")))
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "drone": [0, 0, 1, 0, 0, 0], "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
for i in range(30):
    e.step(np.array(sd, np.float64))
print(model, K, H, "block_threads", bt or "default", flush=True)
e.close()
