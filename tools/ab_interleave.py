"""Interleaved same-process A/B of library builds (tools/, not shipped).

    python tools/ab_interleave.py <reps> "<model K H [V nb threads [full]]>;..." lib_a.so lib_b.so ...

Every build is loaded into the one process (RTLD_LOCAL, its own kernels), an engine per
(build, workload) is created up front, and the builds' kernel timings alternate rep by
rep, so clock and thermal drift hit every build alike.  Prints per build and workload the
median and the inter-quartile range of the back-to-back rollout and finalize times and of
the (rollout, finalize) pair."""
import ctypes as C
import os
import sys

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
    libs = sys.argv[3:]
    handles = [load(p) for p in libs]
    eng = {}
    for li, h in enumerate(handles):
        capi._lib = h
        for ri, r in enumerate(runs):
            model, K, H = r[0], int(r[1]), int(r[2])
            V = int(r[3]) if len(r) > 3 else 1
            nb = int(r[4]) if len(r) > 4 else 0
            th = int(r[5]) if len(r) > 5 else 0
            kw = {}
            if len(r) > 6 and r[6] == "full":   # a full Sigma: the extended (XC) kernel
                A = {"drone": 3, "arm": 7, "wholebody": 10}[model]
                sig = np.eye(A, dtype=np.float32) * 0.1
                sig[0, 1] = sig[1, 0] = 0.02
                kw["sigma"] = sig
            e = Engine(make_config(model, n_samples=K, n_horizon=H, n_vehicles=V, blocks_per_vehicle=nb,
                                   block_threads=th, state_f64=(model == "arm"), **kw))
            for v in range(V):
                if model in ("drone", "quadrotor"):
                    e.set_target([1.0, 2.0, 3.4], vehicle=v)
                else:
                    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5], vehicle=v)
            e.set_state(np.tile(np.array(STATE[model], np.float64), (V, 1)))
            e.run_steps(20)
            e.synchronize()
            eng[li, ri] = e
    res = {k: [] for k in eng}
    for rep in range(reps):
        for ri in range(len(runs)):
            for li in range(len(handles)):
                e = eng[li, ri]
                has_ex = hasattr(handles[li], "mppi_kernel_timing_ex")
                if has_ex:
                    r, f, p = e.kernel_timing_ex(100)
                else:
                    (r, f), p = e.kernel_timing(100), float("nan")
                res[li, ri].append((r, f, p))
    for ri, r in enumerate(runs):
        print(" ".join(r), flush=True)
        for li, path in enumerate(libs):
            a = np.array(res[li, ri])
            q = np.percentile(a, [25, 50, 75], axis=0)
            gbs = eng[li, ri].rollout_bytes() / q[1, 0] / 1e3
            print(f"  {os.path.basename(path):18s} rollout {q[1, 0]:7.2f} [{q[0, 0]:6.2f},{q[2, 0]:6.2f}] us "
                  f"finalize {q[1, 1]:6.2f} pair {q[1, 2]:7.2f} us  rollout {gbs:7.1f} GB/s", flush=True)
    for e in eng.values():
        e.close()


if __name__ == "__main__":
    main()
