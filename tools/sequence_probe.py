"""Kernel-sequence timing (tools/, MPPI_PROBE builds only): what a (rollout, X) pair costs for
X = an empty kernel, a one-block rollout (same kernel object), the finalize.

    MPPI_HIP_LIB=abl/probe.so python tools/sequence_probe.py   (GPU)"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

NAMES = ["rollout+empty", "rollout+rollout(1 block)", "rollout+finalize", "empty", "rollout(1 block)", "rollout"]
for model, K, H, f64 in (("arm", 4096, 32, True), ("wholebody", 8192, 64, False)):
    e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=f64))
    sd = [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * (7 if model == "arm" else 10)
    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5]); e.set_state(np.array(sd, np.float64))
    e.run_steps(100); e.synchronize()
    fn = e._L.mppi_probe_sequence
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_double)]
    res = {}
    for rep in range(5):
        for m in range(6):
            us = C.c_double()
            fn(e._h, 200, m, C.byref(us))
            res.setdefault(m, []).append(us.value)
    print(model, K, H, "  ".join(f"{NAMES[m]} {np.median(v):.2f}" for m, v in res.items()), flush=True)
    e.close()
