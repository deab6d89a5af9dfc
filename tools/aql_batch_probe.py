"""Short-batch cost of native vs HIP dispatch (tools/): median wall time of
`run_steps(n); synchronize()` for n = 1..200, after an untimed priming batch each time, so
the intercept is the per-batch bracket (first kernel start + completion wake-up) and the
slope the per-step time."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (the bench's process shape: torch's HIP runtime loaded first)

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
ST = np.array([0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7, np.float64)


def mk(mode):
    os.environ["MPPI_DISPATCH"] = mode
    e = Engine(make_config("arm", device=0, seed=3, n_samples=4096, n_horizon=32, state_f64=True))
    e.set_target([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
    e.set_state(ST)
    e.run_steps(50)
    e.synchronize()
    return e


engines = {m: mk(m) for m in ("hip", "aql")}
ns = [1, 2, 5, 10, 20, 50, 200]
res = {m: {} for m in engines}
for rep in range(15):
    for m, e in engines.items():
        for n in ns:
            e.run_steps(10)   # priming, untimed
            e.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.run_steps(n)
            t1 = time.perf_counter()
            e.synchronize()
            ts = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            e.synchronize()          # both again, idle: the bracket's own host cost
            ti = time.perf_counter()
            torch.cuda.synchronize()
            tj = time.perf_counter()
            res[m].setdefault(n, []).append(((t2 - t0) * 1e6, (t1 - t0) * 1e6, (ts - t1) * 1e6, (t2 - ts) * 1e6,
                                             (ti - t2) * 1e6, (tj - ti) * 1e6))
for m in engines:
    tot = [np.median([x[0] for x in res[m][n]]) for n in ns]
    enq = [np.median([x[1] for x in res[m][n]]) for n in ns]
    slope, icpt = np.polyfit(ns, tot, 1)
    print(f"{m}: " + "  ".join(f"n={n}: {t:.1f} us (enq {q:.1f})" for n, t, q in zip(ns, tot, enq)) +
          f"  | fit: {slope:.2f} us/step + {icpt:.1f} us per batch; n=20 -> {tot[ns.index(20)] / 20:.2f} us/step")
    for n in (1, 20):
        med = np.median(np.array(res[m][n]), axis=0)
        print(f"  {m} n={n}: run_steps call {med[1]:.1f}, engine sync {med[2]:.1f}, torch sync {med[3]:.1f} us; "
              f"idle: engine sync {med[4]:.1f}, torch sync {med[5]:.1f} us")
