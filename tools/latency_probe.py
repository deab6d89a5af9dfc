"""Control-call latency breakdown (host-inclusive, what compute_control_input sees):
enqueue (set_state + rollout + finalize calls) vs wait (read_outputs), for the
completion-flag poll (default) and the output-event wait (MPPI_EVENT_WAIT=1).

    python tools/latency_probe.py [arm|drone|wholebody] [K] [H]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

model = sys.argv[1] if len(sys.argv) > 1 else "arm"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
H = int(sys.argv[3]) if len(sys.argv) > 3 else 32
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "drone": [0, 0, 1, 0, 0, 0],
      "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
state = np.array(sd, np.float64)
n = 400
for mode in ("flag", "event"):
    if mode == "event":
        os.environ["MPPI_EVENT_WAIT"] = "1"
    else:
        os.environ.pop("MPPI_EVENT_WAIT", None)
    e = Engine(make_config(model, n_samples=K, n_horizon=H, state_f64=(model == "arm")))
    e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
    for _ in range(50):
        e.step(state)
    full, enq, wait = [], [], []
    for _ in range(n):
        t0 = time.perf_counter()
        e.step(state)
        full.append(time.perf_counter() - t0)
    for _ in range(n):
        t0 = time.perf_counter()
        e.set_state(state)
        e.rollout()
        e.finalize()
        t1 = time.perf_counter()
        e.read_outputs()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        wait.append(t2 - t1)
    q = lambda x, p: np.percentile(np.array(x) * 1e6, p)
    print(f"{model} K={K} H={H} wait={mode}: step p50 {q(full, 50):6.1f} us p99 {q(full, 99):6.1f} | split: "
          f"enqueue p50 {q(enq, 50):5.1f} us, read_outputs p50 {q(wait, 50):5.1f} us", flush=True)
    e.close()
