"""Interleaved same-process A/B of library builds on the NATIVE dispatch path (tools/, not shipped).

    python tools/ab_native.py <reps> "<model K H [V]>;..." lib_a.so lib_b.so[@VAR=value,...] ...

A build may carry environment settings read at engine creation (lib.so@MPPI_FUSED=0): they are
set while that build's engines are created.

Each build is loaded into the one process (RTLD_LOCAL; its code objects next to it), one engine
per (build, workload); per rep and build: a 50-step priming batch, then the wall time of a
`steps` batch (default 500, MPPI_AB_STEPS) and of 20 control calls (MPPI_AB_CALLS).  Prints the median us per
step and per call and their inter-quartile ranges."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd import _capi as capi
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

STATE = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
         "drone": [0, 0, 1, 0, 0, 0], "quadrotor": [0, 0, 1, 0, 0, 0] + [0.0] * 6,
         "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}


def load(path):
    h = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
    for name, (res, args) in capi.PROTOTYPES.items():
        if hasattr(h, name):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
    return h


def main():
    reps = int(sys.argv[1])
    runs = [r.split() for r in sys.argv[2].split(";") if r.strip()]
    # (the engines below index the runs by position; "peer" is stripped per run there)
    libs = sys.argv[3:]
    steps = int(os.environ.get("MPPI_AB_STEPS", "500"))
    ncalls = int(os.environ.get("MPPI_AB_CALLS", "20"))   # 0 for builds without completion flags (knockouts)
    eng = {}
    for li, spec in enumerate(libs):
        p, _, envs = spec.partition("@")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        capi._lib = load(p)
        for ri, r in enumerate(runs):
            peer = "peer" in r   # "<model K H peer>": one rank exchanging with itself (the C4 rank's step)
            r = [x for x in r if x != "peer"]
            model, K, H = r[0], int(r[1]), int(r[2])
            V = int(r[3]) if len(r) > 3 else 1
            e = Engine(make_config(model, n_samples=K, n_horizon=H, n_vehicles=V, state_f64=(model == "arm")))
            if peer:
                e.peer_connect([e.peer_open()])
                for ph in (0, 1, 2):
                    e.peer_probe(ph)
            for v in range(V):
                if model in ("drone", "quadrotor"):
                    e.set_target([1.0, 2.0, 3.4], vehicle=v)
                else:
                    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
            e.set_state(np.tile(np.array(STATE[model], np.float64), (V, 1)))
            e.run_steps(20)
            e.synchronize()
            eng[li, ri] = e
        for k, val in saved.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val
    res = {k: [] for k in eng}
    for rep in range(reps):
        for ri, r in enumerate(runs):
            st = np.tile(np.array(STATE[r[0]], np.float64), (eng[0, ri].V, 1))
            for li in range(len(libs)):
                e = eng[li, ri]
                e.run_steps(50)
                e.synchronize()
                t0 = time.perf_counter()
                e.run_steps(steps)
                e.synchronize()
                t1 = time.perf_counter()
                calls = [0.0]
                for _ in range(ncalls):
                    c0 = time.perf_counter()
                    e.step(st)
                    calls.append(time.perf_counter() - c0)
                res[li, ri].append(((t1 - t0) / steps * 1e6, float(np.median(calls)) * 1e6))
    for ri, r in enumerate(runs):
        print(" ".join(r), flush=True)
        for li, path in enumerate(libs):
            a = np.array(res[li, ri])
            q = np.percentile(a, [25, 50, 75], axis=0)
            print(f"  {os.path.relpath(path):26s} step {q[1, 0]:7.2f} [{q[0, 0]:6.2f},{q[2, 0]:6.2f}] us   "
                  f"call {q[1, 1]:6.2f} [{q[0, 1]:6.2f},{q[2, 1]:6.2f}] us   ({eng[li, ri].dispatch_info()})", flush=True)
    for e in eng.values():
        e.close()


if __name__ == "__main__":
    main()
