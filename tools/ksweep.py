"""Rollout/finalize kernel time vs K (rocprof-independent, HIP events)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
model = sys.argv[1] if len(sys.argv) > 1 else "arm"
H = int(sys.argv[2]) if len(sys.argv) > 2 else 32
res = []
KS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536]
for K in KS:
    e = Engine(make_config(model, n_samples=K, n_horizon=H))
    sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
          "drone": [0, 0, 1, 0, 0, 0], "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(np.array(sd, np.float64))
    e.run_steps(20); e.synchronize()
    r, f = e.kernel_timing(300)
    res.append((K, r, f, e.rollout_bytes()))
    print(f"K={K:6d} H={H} rollout {r:8.2f} us  finalize {f:6.2f} us  GB/s {e.rollout_bytes()/r/1e3:8.1f}", flush=True)
    e.close()
