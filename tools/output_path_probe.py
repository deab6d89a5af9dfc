"""Where a back-to-back control step loses time against the kernel-timing pair (tools/).

    python tools/output_path_probe.py [workload] [steps]

One process per MPPI_DEBUG_OUT setting (0: production; 1: unread steps write their
outputs to device scratch; 2: mppi_kernel_timing writes to mapped host memory): the
event-timed (rollout, finalize) pair of mppi_kernel_timing_ex, and batches of
mppi_run_steps timed with torch events on the engine stream (GPU time) and on the host
(enqueue, wall)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    placement = os.environ.get("MPPI_PROBE_CPUS")   # local | remote | unset (the box's default)
    if placement:
        from quadrotor_manipulator_mppi_amd.affinity import gpu_local_cpus
        local = set(gpu_local_cpus(0) or [])
        cur = set(os.sched_getaffinity(0))
        want = (cur & local) if placement == "local" else (cur - local)
        if want:
            os.sched_setaffinity(0, sorted(want))
    import torch
    import bench
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    name = sys.argv[1] if len(sys.argv) > 1 else "arm_c3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    w = dict(bench.WORKLOADS[name])
    w.pop("desc")
    w.pop("strong", None)
    native = w.pop("native", None)
    se = ShardedEngine(seed=1234, native=native, **w)
    eng = se.engine
    bench.set_targets(eng, w["model"], w.get("n_vehicles", 1))
    eng.set_state(bench.make_state(w["model"], w.get("n_vehicles", 1)))
    se.run_steps(100)
    eng.synchronize()
    pairs = [eng.kernel_timing_ex(200)[2] for _ in range(5)]
    rows = []
    pause = float(os.environ.get("MPPI_PROBE_PAUSE_MS", "0")) * 1e-3   # host pause after each batch's sync
    spin = float(os.environ.get("MPPI_PROBE_SPIN_MS", "0")) * 1e-3     # host busy loop after each batch's sync
    for _ in range(12):
        eng.synchronize()
        torch.cuda.synchronize()
        if pause:
            time.sleep(pause)
        if spin:   # busy host before the batch (CPU frequency hypothesis)
            t_end = time.perf_counter() + spin
            while time.perf_counter() < t_end:
                pass
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(se.stream)
        se.run_steps(steps)
        e1.record(se.stream)
        t1 = time.perf_counter()
        eng.synchronize()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows.append((e0.elapsed_time(e1) * 1e3 / steps, (t1 - t0) * 1e6 / steps, (t2 - t0) * 1e6 / steps))
    a = np.array(rows)
    print(json.dumps({"workload": name, "steps": steps, "MPPI_DEBUG_OUT": os.environ.get("MPPI_DEBUG_OUT", "0"),
                      "cpus": os.environ.get("MPPI_PROBE_CPUS", "default"), "ncpus": len(os.sched_getaffinity(0)),
                      "pause_ms": pause * 1e3, "spin_ms": spin * 1e3,
                      "enqueue_batches": [round(x, 2) for x in a[:, 1]],
                      "pair_us": round(float(np.median(pairs)), 3),
                      "run_steps_gpu_us": round(float(np.median(a[:, 0])), 3),
                      "run_steps_enqueue_us": round(float(np.median(a[:, 1])), 3),
                      "run_steps_wall_us": round(float(np.median(a[:, 2])), 3)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
