"""Same-process A/B of the host-side control-call path (tools/, not shipped).

    python tools/latency_ab.py        (GPU)

Arm C3 engine; alternating batches of 200 ``Engine.step`` calls with the state as a flat
float64 array (the one-slice-copy fast path) and as a (1, 21) array (the reshape path, the
previous per-call copy), median per-call latency of each over 10 batches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

e = Engine(make_config("arm", n_samples=4096, n_horizon=32, state_f64=True))
e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
flat = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
two_d = flat.reshape(1, -1).copy()
res = {"flat": [], "2d": []}
for _ in range(50):
    e.step(flat)
for b in range(10):
    for name, s in (("flat", flat), ("2d", two_d)) if b % 2 == 0 else (("2d", two_d), ("flat", flat)):
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            e.step(s)
            ts.append(time.perf_counter() - t0)
        res[name].append(np.median(ts) * 1e6)
for name, v in res.items():
    print(f"{name:5s} per-call p50 over batches: median {np.median(v):.2f} us  (min {min(v):.2f}, max {max(v):.2f})")
e.close()
