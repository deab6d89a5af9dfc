"""Interleaved same-process A/B of rollout launch geometries on the native path (tools/, not shipped):
    python tools/ab_geometry.py <reps> "<model K H>;..." <threads[:blocks]> <threads[:blocks]> ...
(blocks = blocks per vehicle, 0 = the engine's automatic choice).  One engine per (workload,
geometry); per rep, in alternating order: a 50-step priming batch, then the wall time of a
500-step batch.  Prints the median us per step and its IQR."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

STATE = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
         "drone": [0, 0, 1, 0, 0, 0],
         "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}


def main():
    reps = int(sys.argv[1])
    runs = [r.split() for r in sys.argv[2].split(";") if r.strip()]
    sizes = [tuple(int(y) for y in (x.split(":") + ["0"])[:2]) for x in sys.argv[3:]]
    eng = {}
    for r in runs:
        model, K, H = r[0], int(r[1]), int(r[2])
        for t in sizes:
            e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=(model == "arm"), block_threads=t[0],
                                   blocks_per_vehicle=t[1]))
            if model == "drone":
                e.set_target([1.0, 2.0, 3.4])
            else:
                e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
            e.set_state(np.array(STATE[model], np.float64))
            e.run_steps(20)
            e.synchronize()
            eng[r[0], t] = e
    res = {k: [] for k in eng}
    for rep in range(reps):
        order = sizes if rep % 2 == 0 else sizes[::-1]
        for r in runs:
            for t in order:
                e = eng[r[0], t]
                e.run_steps(50)
                e.synchronize()
                t0 = time.perf_counter()
                e.run_steps(500)
                e.synchronize()
                res[r[0], t].append((time.perf_counter() - t0) / 500 * 1e6)
    for r in runs:
        print(" ".join(r))
        for t in sizes:
            q = np.percentile(res[r[0], t], [25, 50, 75])
            print(f"  threads {t[0]:4d} blocks {t[1] or 'auto':>4}  step {q[1]:7.2f} [{q[0]:6.2f},{q[2]:6.2f}] us  "
                  f"({eng[r[0], t].dispatch_info()})")
    for e in eng.values():
        e.close()


if __name__ == "__main__":
    main()
