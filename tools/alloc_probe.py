"""Does a buffer's allocation order change the rollout time?  N identical engines,
timings interleaved (tools/, not shipped).   python tools/alloc_probe.py N reps [pre_mb]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

n, reps = int(sys.argv[1]), int(sys.argv[2])
pre = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if pre:   # occupy some device memory first (torch's allocator) to shift the engines' placement
    hold = torch.empty(pre << 20, dtype=torch.uint8, device="cuda")
st = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10, np.float64)
engs = []
for i in range(n):
    e = Engine(make_config("wholebody", n_samples=8192, n_horizon=64, blocks_per_vehicle=512))
    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(st)
    e.run_steps(20)
    e.synchronize()
    engs.append(e)
res = [[] for _ in engs]
for r in range(reps):
    for i, e in enumerate(engs):
        res[i].append(e.kernel_timing(100)[0])
for i in range(n):
    a = np.array(res[i])
    print(f"engine {i}: rollout median {np.median(a):.2f} us [{np.percentile(a, 25):.2f}, {np.percentile(a, 75):.2f}]")
