"""Where a native control call's host time goes (tools/): p50 of (a) the bare C entry point
mppi_step through ctypes with preset pointers, (b) Engine.step (numpy staging, copies, stats
objects), (c) the drop-in MPPI.compute_control_input, at C3 with a changing state."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from quadrotor_manipulator_mppi_amd import _capi as capi
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
ST = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, np.float64)
e = Engine(make_config("arm", device=0, seed=3, n_samples=4096, n_horizon=32, state_f64=True))
e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
e.set_state(ST)
L = capi.lib()
rng = np.random.default_rng(0)
states = [ST + np.r_[np.zeros(7), rng.normal(0, 0.01, 7), np.zeros(7)] for _ in range(64)]


def p50(f, n=3000):
    ts = []
    for i in range(n):
        t0 = time.perf_counter()
        f(i)
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts[200:]) * 1e6
    return np.median(ts), np.percentile(ts, 99)


st_buf = np.zeros(21, np.float64)
p_state = st_buf.ctypes.data_as(C.POINTER(C.c_double))
out = np.zeros((1, e.out_dim), np.float64)
u0 = np.zeros((1, e.A), np.float32)
stats = (capi.Stats * 1)()
p_out = out.ctypes.data_as(C.POINTER(C.c_double))
p_u0 = u0.ctypes.data_as(C.POINTER(C.c_float))


def bare(i):
    st_buf[:] = states[i & 63]
    L.mppi_step(e._h, p_state, None, p_out, p_u0, stats)


def eng(i):
    e.step(states[i & 63])


print("bare C mppi_step     p50 %.2f us  p99 %.2f" % p50(bare))
print("Engine.step          p50 %.2f us  p99 %.2f" % p50(eng))
print("bare C mppi_step     p50 %.2f us  p99 %.2f" % p50(bare))
print("dispatch:", e.dispatch_info())
from quadrotor_manipulator_mppi_amd.mppi_solver.mppi import MPPI
m = MPPI(n_samples=4096)
q_full = np.array([0, 0, 1, 0, 0, 0, 1] + HOME, np.float64)
v_full = np.zeros(13, np.float64)


def dropin(i):
    q_full[7:14] = states[i & 63][7:14]
    m.update_joint(q_full, v_full)
    m.compute_control_input()


print("MPPI.compute_control_input (update_joint + call)  p50 %.2f us  p99 %.2f" % p50(dropin))
