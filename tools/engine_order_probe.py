"""Per-step time of three identical engines created one after another in one process (tools/, not shipped)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}
for model, K, H, V in (("arm", 4096, 32, 1), ("wholebody", 8192, 64, 1), ("wholebody", 8192, 64, 8)):
    es = []
    for i in range(3):
        e = Engine(make_config(model, n_samples=K, n_horizon=H, n_vehicles=V, state_f64=(model == "arm")))
        for v in range(V): e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
        e.set_state(np.tile(np.array(sd[model], np.float64), (V, 1))); e.run_steps(50); e.synchronize()
        es.append(e)
    res = [[] for _ in es]
    for rep in range(7):
        for i, e in enumerate(es):
            t0 = time.perf_counter(); e.run_steps(500); e.synchronize(); res[i].append((time.perf_counter() - t0) / 500 * 1e6)
    print(model, V, K, H, "engine order 1/2/3 us/step:", [round(float(np.median(r)), 2) for r in res], flush=True)
    for e in es: e.close()
