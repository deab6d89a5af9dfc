"""Launch-geometry sweep: rollout/finalize kernel time and back-to-back step time
vs blocks per vehicle (iters = groups/nb) and block size.
   python tools/geom_sweep.py wholebody 8192 64 [nb,nb,...] [threads,...]"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
model, K, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
NBS = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
THS = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [0]
V = int(os.environ.get("GEOM_V", "1"))
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "drone": [0, 0, 1, 0, 0, 0], "quadrotor": [0, 0, 1, 0, 0, 0] + [0.0] * 6, "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
for th in THS:
    for nb in NBS:
        e = Engine(make_config(model, n_samples=K, n_horizon=H, n_vehicles=V, blocks_per_vehicle=nb,
                               block_threads=th, state_f64=(model == "arm")))
        for v in range(V):
            e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
        e.set_state(np.tile(np.array(sd, np.float64), (V, 1)))
        e.run_steps(50); e.synchronize()
        n = 1000
        t0 = time.perf_counter(); e.run_steps(n); e.synchronize(); dt = time.perf_counter() - t0
        r, f = e.kernel_timing(300)
        print(f"{model} V={V} K={K} H={H} threads={th or 'dflt'} nb={e.dp_nb() if hasattr(e, 'dp_nb') else nb}: "
              f"step {dt / n * 1e6:7.2f} us  rollout {r:7.2f} us  finalize {f:6.2f} us  "
              f"rollout GB/s {e.rollout_bytes() / r / 1e3:7.1f}", flush=True)
        e.close()
