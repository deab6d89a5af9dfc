"""Control-call latency, native vs HIP dispatch (tools/): p50/p90 of Engine.step at C3 with a
changing state, n calls per mode, modes interleaved in blocks of 200."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
ST = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, np.float64)
modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["hip", "aql"]
eng = {}
for m in modes:
    os.environ["MPPI_DISPATCH"] = m
    e = Engine(make_config("arm", device=0, seed=3, n_samples=4096, n_horizon=32, state_f64=True))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(ST)
    eng[m] = e
rng = np.random.default_rng(0)
lat = {m: [] for m in modes}
for blk in range(10):
    for m, e in eng.items():
        for i in range(220):
            st = ST.copy()
            st[7:14] += rng.normal(0, 0.01, 7)
            t0 = time.perf_counter()
            e.step(st)
            if i >= 20:
                lat[m].append((time.perf_counter() - t0) * 1e6)
for m in modes:
    x = np.array(lat[m])
    print(f"{m}: calls {eng[m].dispatch_info()!r}  p50 {np.median(x):.2f} us  p10 {np.percentile(x, 10):.2f}  "
          f"p90 {np.percentile(x, 90):.2f}  p99 {np.percentile(x, 99):.2f}")
