"""Joint-angle error of the fp32 integrator against the oracle's fp64-state cumsums
(standard_normal_noise.py:41-48 after the float64 promotion of mppi.py:197).

    python tools/integrator_error.py        (GPU; prints one line per shape)

The engine integrates the increments in fp32 (transposed LDS integrator for H <= 64,
DPP segment scans for H > 64) and adds q0 in the state dtype; the oracle accumulates in
the state dtype.  This prints max |q_gpu - q_oracle| over all (k, t, joint) for fp64
state, with nonzero joint rates and a nonzero warm start, i.e. the number DESIGN.md §5
quotes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import mppi_oracle as O
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
from quadrotor_manipulator_mppi_amd.robot.urdf_chain import load_chain

chain = [O.Joint(j["name"], j["type"], j["xyz"], j["rpy"], j["axis"], j["q_index"]) for j in load_chain()]
TP, TQ = [0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5]
for H in (16, 32, 64, 100, 128):
    K = 512
    torch.manual_seed(7 + H)
    noise = O.draw_noise(K, H, torch.eye(7) * 0.1)
    u_prev = torch.randn(H, 7) * 0.3
    q_full = np.array([0.1, -0.2, 1.1, 0.0, 0.0, 0.2588190, 0.9659258] + [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0])
    v_full = np.array([0.0] * 6 + [0.8, -0.5, 0.3, -1.2, 0.4, 0.9, -0.7])
    r = O.arm_step(chain, q_full, v_full, u_prev, noise, TP, TQ, f64=True)
    e = Engine(make_config(model="arm", n_samples=K, n_horizon=H, noise="injected", state_f64=True))
    e.set_target(TP, TQ)
    e.set_u_prev(u_prev.numpy())
    e.step(np.concatenate([q_full[:7], q_full[7:], v_full[6:]]), noise.numpy()[None])
    q = e.get_trajectory()[0][..., :7].astype(np.float64)
    ref = r["q_samples"].numpy().astype(np.float64)
    err = np.abs(q - ref)
    err32 = np.abs(q - ref.astype(np.float32).astype(np.float64))   # beyond the fp32 trajectory storage
    rng = np.abs(ref - q_full[7:]).max()
    print(f"arm fp64 state K={K} H={H}: max |dq| = {err.max():.3e} rad (mean {err.mean():.2e}; "
          f"vs the fp32-rounded oracle {err32.max():.3e}, "
          f"{np.count_nonzero(err32) / err32.size:.1%} of entries differ); "
          f"max |q - q0| over the horizon {rng:.3f} rad; fp32 ulp at |q|<=8: {np.spacing(np.float32(8)):.2e}",
          flush=True)
    e.close()
