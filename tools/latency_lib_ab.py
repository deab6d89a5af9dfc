"""Same-process A/B of library builds on the host-inclusive control call (tools/).

    python tools/latency_lib_ab.py <reps> lib_a.so lib_b.so ...

One arm C3 engine per build (K=4096 H=32, fp64 state, the bench's state and target);
alternating batches of 200 ``Engine.step`` calls (set_state, rollout, finalize, the
completion-flag wait, outputs, check_reach), the order rotating per rep; prints each
build's median per-call latency and its p10/p90 over all calls."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ab_interleave import load
from quadrotor_manipulator_mppi_amd import _capi as capi
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config


def main():
    reps = int(sys.argv[1])
    libs = sys.argv[2:]
    state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
    engs = []
    for path in libs:
        capi._lib = load(path)
        e = Engine(make_config("arm", n_samples=4096, n_horizon=32, state_f64=True))
        e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
        for _ in range(50):
            e.step(state)
        engs.append(e)
    res = [[] for _ in libs]
    for rep in range(reps):
        order = list(range(len(libs)))
        order = order[rep % len(order):] + order[:rep % len(order)]
        for li in order:
            e = engs[li]
            for _ in range(200):
                t0 = time.perf_counter()
                e.step(state)
                res[li].append(time.perf_counter() - t0)
    for li, path in enumerate(libs):
        a = np.array(res[li]) * 1e6
        print(f"{os.path.basename(path):18s} control call p50 {np.median(a):6.2f} us  p10 {np.percentile(a, 10):6.2f}  "
              f"p90 {np.percentile(a, 90):6.2f}  ({a.size} calls)", flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
